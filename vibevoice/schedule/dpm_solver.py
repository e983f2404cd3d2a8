"""Reference path vibevoice/schedule/dpm_solver.py: the scheduler object behind
`model.model.noise_scheduler` (its `.from_config(config, algorithm_type=...,
beta_schedule=...)` swap, gradio_demo.py:114-118).  The per-step arithmetic
runs on the device (k_cfg_dpm); this class builds its coefficient tables."""
from vibevoice_amd.schedule import Schedule as DPMSolverMultistepScheduler  # noqa: F401

__all__ = ["DPMSolverMultistepScheduler"]
