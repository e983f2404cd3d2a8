"""Teacher-forced full-size parity (shared by test_gpu_fullsize.py and
test_gpu_large_e2e.py).

The oracle (oracle/loop.py, pinned to the reference's own generate() by golden
G8) runs the loop in bf16 — the reference's GPU dtype — and records each
step's inputs.  The product loop is then driven with exactly those inputs: the
prompt embeddings, every step's next input embedding and, for the codec, every
step's latent.  Each step's outputs therefore measure one step of arithmetic,
not accumulated autoregressive drift:

  hpos / hneg   positive / negative final-norm hidden states (LM pass)
  logits        the 4 legal logits the constrained argmax reads (:494-507)
  latents       the CFG DPM-Solver++ diffusion output (sample_speech_tokens)
  audio         the streaming acoustic-decoder chunk (3,200 samples)
  next          the next step's input embedding of the diffusing rows: the
                acoustic connector of the latent + the semantic connector of
                the streaming semantic encoding of the audio (:673-687)

Bounds are FIXED per quantity (rel L2 per step, stated in DESIGN.md §4), near
what is measured.  Where the fp32 oracle run is given, each quantity's worst
error is ALSO tied to the bf16 reference's own noise: worst rel <= NOISE_C x
max(the bf16 reference's worst deviation from fp32 on the same inputs,
NOISE_FLOOR), so a regression that stays under the fixed bound but well above
the reference's own bf16 noise fails (round-4 parity log, profiles/r04_parity.log:
the largest ratio is 1.8, the S = 5 logits).
"""
import torch

from gpu_util import rel_err
from oracle import loop as oloop

dev = "cuda"
# fixed per-step rel-L2 bounds (measured worst over the 1.5B B=1 S=10/5, B=8 and
# Large 4-speaker runs, round 3: hidden 2.25e-2, next-step embeddings 2.0e-2,
# audio 1.6e-2, logits 5.0e-2, latents 5.2e-2)
BOUND = dict(hpos=3e-2, hneg=3e-2, latents=7e-2, audio=3e-2, logits=7e-2, next=3e-2)
NOISE_C, NOISE_FLOOR = 2.5, 5e-3


def oracle_run(sd, cfg, inp, sched, ids, steps, vn, seed, dtype=torch.bfloat16, teacher=None, max_new=None):
    rec = {}
    torch.manual_seed(seed)
    seqs, audio, reach = oloop.generate(sd, cfg, inp["input_ids"], inp["attention_mask"], ids, ddpm_steps=steps,
                                        cfg_scale=1.3, forced=sched, dtype=dtype, record=rec, voice_noise=vn,
                                        teacher=teacher, max_new_tokens=max_new,
                                        speech_tensors=inp["speech_tensors"], speech_masks=inp["speech_masks"],
                                        speech_input_mask=inp["speech_input_mask"])
    return rec, seqs, audio, reach


def teacher_forced(model, inp, sched, rec, tok, seed, max_new=None):
    """Drive the product loop with the oracle run's inputs.  Returns the
    per-step outputs the product computed, and the session.  max_new: the
    oracle run's max_new_tokens when its length cap ended it."""
    B = inp["input_ids"].shape[0]
    got = dict(hpos=[], hneg=[], logits=[], latents=[], audio=[], next=[])
    pe = rec["prompt_embeds"].to(dev, torch.bfloat16)
    orig = model._prompt_embeds
    model._prompt_embeds = lambda *a, **k: pe.clone()
    try:
        torch.manual_seed(seed)
        sess = model.generate_session(input_ids=inp["input_ids"], attention_mask=inp["attention_mask"], tokenizer=tok,
                                      cfg_scale=1.3, forced_tokens=sched, show_progress_bar=False,
                                      max_new_tokens=max_new or max(len(s) for s in sched) + 2)
    finally:
        model._prompt_embeds = orig
    post = sess._post_phase

    def hooked(n):
        k = sess.step_idx
        got["hpos"].append(sess.hid[:B].float().cpu())
        got["hneg"].append(sess.hid[B:].float().cpu())
        got["logits"].append(sess.logits_pin.clone()[:, sess.order])          # sorted ids, as the oracle records
        if n:
            got["latents"].append(sess.noise_dev[:n].float().cpu())
            sess.noise_dev[:n].copy_(rec["latents"][len(got["latents"]) - 1].to(dev, torch.bfloat16))
        post(n)
        if n:
            got["audio"].append(sess.audio_dev[:n].float().cpu())
        got["next"].append(sess.x_in2[:B].float().cpu())                      # before the teacher overwrites it
        sess.x_in2[:B].copy_(rec["next_embeds"][k].to(dev, torch.bfloat16))
    sess._post_phase = hooked
    while sess.step():
        pass
    torch.cuda.synchronize()
    return got, sess


def per_step_check(got, rec16, rec32, tag, bound=BOUND):
    """rel L2 per step and quantity vs the bf16 oracle, against the fixed
    bounds; rec32 (the fp32 oracle teacher-forced on the bf16 run, or None) is
    only printed, for scale."""
    worst, fails = {}, []
    dsteps = [k for k, d in enumerate(rec16["didx"]) if d.numel()]

    def one(q, j, g, r, r32):
        e = rel_err(g, r)
        sdev = rel_err(r32, r) if r32 is not None else float("nan")
        if e > worst.get(q, (-1.0,))[0]:
            worst[q] = (e, sdev)
        if not e < bound[q]:
            fails.append(f"{q}[{j}] rel {e:.3e} >= {bound[q]:.1e} (bf16 reference self-deviation {sdev:.3e})")

    nsteps = len(rec16["hpos"])
    assert len(got["hpos"]) == nsteps, (len(got["hpos"]), nsteps)
    for j in range(nsteps):
        r32 = rec32["hpos"][j] if rec32 else None
        one("hpos", j, got["hpos"][j], rec16["hpos"][j], r32)
        one("logits", j, got["logits"][j], rec16["logits"][j], rec32["logits"][j] if rec32 else None)
        rows = rec16["didx"][j]
        if j in dsteps and rec16["hneg"][j] is not None:        # the negative rows the head consumes
            one("hneg", j, got["hneg"][j][rows], rec16["hneg"][j][rows],
                rec32["hneg"][j][rows] if rec32 else None)
        if rows.numel():                                           # connectors of the diffusing rows
            one("next", j, got["next"][j][rows], rec16["next_embeds"][j][rows],
                rec32["next_embeds"][j][rows] if rec32 else None)
    assert len(got["latents"]) == len(rec16["latents"]) == len(dsteps)
    for j in range(len(dsteps)):
        for q in ("latents", "audio"):
            r = rec16[q][j]
            one(q, j, got[q][j].reshape(r.shape), r, rec32[q][j] if rec32 else None)
    sworst = {}
    for q, (e, sd_) in sorted(worst.items()):
        print(f"{tag} {q}: worst rel {e:.3e} (bound {bound[q]:.1e}; bf16 reference self-deviation {sd_:.3e})")
    if rec32 is not None:
        # the reference's own worst bf16 deviation per quantity (over all steps)
        for j in range(nsteps):
            rows = rec16["didx"][j]
            pairs = [("hpos", rec16["hpos"][j], rec32["hpos"][j]), ("logits", rec16["logits"][j], rec32["logits"][j])]
            if j in dsteps and rec16["hneg"][j] is not None:
                pairs.append(("hneg", rec16["hneg"][j][rows], rec32["hneg"][j][rows]))
            if rows.numel():
                pairs.append(("next", rec16["next_embeds"][j][rows], rec32["next_embeds"][j][rows]))
            for q, r, r32 in pairs:
                sworst[q] = max(sworst.get(q, 0.0), rel_err(r32, r))
        for j in range(len(dsteps)):
            for q in ("latents", "audio"):
                sworst[q] = max(sworst.get(q, 0.0), rel_err(rec32[q][j], rec16[q][j]))
        for q, (e, _) in sorted(worst.items()):
            lim = NOISE_C * max(sworst[q], NOISE_FLOOR)
            print(f"{tag} {q}: worst rel {e:.3e} vs {NOISE_C} x bf16 reference noise {sworst[q]:.3e} = {lim:.3e}")
            if not e <= lim:
                fails.append(f"{q}: worst rel {e:.3e} > {NOISE_C} x the bf16 reference's own worst deviation "
                             f"{sworst[q]:.3e}")
    assert not fails, "\n".join(fails)
    return worst
