"""Debug: per-row audio of the teacher-forced B=8 run (tests/test_gpu_fullsize.py)."""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
import torch
import test_gpu_fullsize as T
from gpu_util import rel_err

m = T.m15.__wrapped__()
D, E, S, X = T.D, T.E, T.S, T.X
inp = T.synthetic_inputs(batch=8, speakers=2, voice_seconds=[3.0, 2.2, 1.3, 2.7], text_tokens=64, seed=101,
                         text_jitter=12)
sched = [[D] * 6 + [X], [D, D, E, S, D, D, X], [D, D, D, X], [S, D, D, D, D, D, X], [D, E, D, D, S, D, X],
         [D, D, D, D, E, S, D, X], [E, S, D, D, D, X], [D, D, S, D, D, D, X]]
vn = T._voice_noise(inp, m.cfg.acoustic_vae_dim)
rec16, seqs, _, reach = T._oracle(m, inp, sched, vn)
for kw in (dict(), dict(use_graphs=False, speculate=False)):
    m.model.use_graphs = kw.get("use_graphs", True)
    got, sess = T._teacher_forced(m.model, inp, sched, rec16)
    print("config", kw)
    for j in range(len(got["audio"])):
        g, r = got["audio"][j], rec16["audio"][j][:, 0]
        print(j, rec16["didx"][[k for k, d in enumerate(rec16["didx"]) if d.numel()][j]].tolist(),
              ["%.2e/%.2f" % (rel_err(g[i], r[i]), g[i].norm() / r[i].norm()) for i in range(g.shape[0])])
