"""The reference's import paths, served by the MI355X engine.

Callers of the reference import `vibevoice.modular.modeling_vibevoice_inference`,
`vibevoice.processor.vibevoice_processor`, `vibevoice.modular.streamer`, ...
(demo/inference_from_file.py:9-10, demo/gradio_demo.py:23-26).  The modules of
this package keep those paths and names and re-export the implementation in
`vibevoice_amd` (HIP engine + host mirror of the reference's interface), so a
demo script runs unchanged with this repository on its PYTHONPATH instead of
the reference.  No arithmetic lives here.
"""
