"""Summarise a rocprofv3 --kernel-trace CSV of `bench.py` per generate-loop step.

Steps are delimited by the restricted lm_head launch (k_final_head, one per LM
pass).  For the last N steps it reports GPU busy time, wall time, idle gap and
the per-kernel (name, grid) breakdown, plus each kernel's average duration.
Usage: python profiles/summarize.py <run_kernel_trace.csv> [n_steps] [out.json]
(out.json: {kernel: {calls_per_step, us_per_step, avg_us}} of those steps -- the
in-loop figures bench.py reports beside its isolated replays.)
"""
import json
import collections
import csv
import re
import sys


def short(name):
    m = re.match(r"_Z(\d+)(\w+)", name)
    if m:                                   # un-demangled (bf16 argument types)
        return m.group(2)[:int(m.group(1))]
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    if "at::native" in n:
        n = "torch:" + n.split("::")[-1][:40]
    return n[:60]


def main(path, n_steps=None, out_json=None):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if r[2] in ("k_lmhead_ids", "k_final_head")]
    steps = list(zip(marks[:-1], marks[1:]))
    # the bench's timed steps are the last ones before the standalone gemv measurement
    if n_steps:
        steps = steps[-n_steps:]
    busy = wall = 0
    per = collections.defaultdict(lambda: [0, 0])
    for a, b in steps:
        seg = rows[a + 1:b + 1]
        wall += rows[b][0] - rows[a + 1][0]
        for s, e, n, g in seg[:-1]:
            busy += e - s
            per[(n, g)][0] += 1
            per[(n, g)][1] += e - s
    k = len(steps)
    print(f"steps {k}: wall/step {wall / k / 1e3:.1f} us, GPU busy/step {busy / k / 1e3:.1f} us, "
          f"launches/step {sum(v[0] for v in per.values()) / k:.0f}")
    byname = collections.defaultdict(lambda: [0, 0])
    for (n, g), (c, t) in per.items():
        byname[n][0] += c
        byname[n][1] += t
    if out_json:
        with open(out_json, "w") as f:
            json.dump({"steps": k, "busy_us_per_step": round(busy / k / 1e3, 1), "wall_us_per_step": round(wall / k / 1e3, 1),
                       "kernels": {n: {"calls_per_step": round(c / k, 2), "us_per_step": round(t / k / 1e3, 2),
                                       "avg_us": round(t / c / 1e3, 3)} for n, (c, t) in byname.items()}}, f, indent=1)
    print(f"{'kernel':60s} {'calls/step':>10s} {'us/step':>9s} {'avg us':>8s}")
    for n, (c, t) in sorted(byname.items(), key=lambda x: -x[1][1]):
        print(f"{n:60s} {c / k:10.1f} {t / k / 1e3:9.1f} {t / c / 1e3:8.2f}")
    print("\nby (kernel, grid), top 30:")
    for (n, g), (c, t) in sorted(per.items(), key=lambda x: -x[1][1])[:30]:
        print(f"{n:40s} {str(g):>16s} {c / k:8.1f}/step {t / k / 1e3:9.1f} us/step  avg {t / c / 1e3:8.2f} us")
    # the last step in launch order (runs of one (kernel, grid) collapsed), with the
    # gap before each launch: where the codec / head / LM phases sit in the step
    a, b = steps[-1]
    seg = rows[a + 1:b + 1]
    print("\nlast step in launch order: start us, kernel, grid, launches x avg us, gap before (us):")
    t0, i = seg[0][0], 0
    while i < len(seg):
        j = i
        while j + 1 < len(seg) and seg[j + 1][2:] == seg[i][2:]:
            j += 1
        run = seg[i:j + 1]
        avg = sum(e - s for s, e, _, _ in run) / len(run) / 1e3
        gap = (seg[i][0] - seg[i - 1][1]) / 1e3 if i else 0.0
        print(f"{(seg[i][0] - t0) / 1e3:9.1f}  {seg[i][2]:40s} {str(seg[i][3]):>16s} {len(run):3d} x {avg:7.2f}  gap {gap:5.2f}")
        i = j + 1


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None, sys.argv[3] if len(sys.argv) > 3 else None)
