"""Per-kernel breakdown of the last prefill rep from a rocprofv3 rocpd database
(rocprofv3 --kernel-trace -d DIR -o pf -- python3 tools/prefill_bench.py L):
python tools/pf_breakdown.py DIR/pf_results.db [reps]"""
import collections
import sqlite3
import sys

db = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, grid_x, grid_y, workgroup_x from kernels order by start").fetchall()
# the prefill reps are separated by the largest gaps between kernels; take the last rep:
# kernels after the last attention-free gap larger than 20 ms
gaps = [(rows[i + 1][1] - rows[i][2], i + 1) for i in range(len(rows) - 1)]
cut = sorted(gaps)[-1][1] if gaps else 0
last = rows[cut:]
tot = collections.defaultdict(lambda: [0, 0.0])
for name, s, e, gx, gy, wx in last:
    k = (name.split("(")[0][:60], gx // max(wx, 1), gy)
    tot[k][0] += 1
    tot[k][1] += (e - s) / 1e3
span = (last[-1][2] - last[0][1]) / 1e6
busy = sum(v[1] for v in tot.values()) / 1e3
print(f"last rep: {len(last)} kernels, span {span:.2f} ms, busy {busy:.2f} ms")
print(f"{'kernel':60s} {'grid':>12s} {'calls':>6s} {'total ms':>9s} {'avg us':>9s}")
for k, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{k[0]:60s} {str((k[1], k[2])):>12s} {n:6d} {us / 1e3:9.3f} {us / n:9.1f}")
