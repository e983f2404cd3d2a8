#!/bin/bash
# decode rate vs context length on one GPU (1.5B, graph-replayed
# decode after a product-path prefill of the prompt).  One bench.py run per
# context, each under its own time limit; stops at the first run that does not
# end normally.  Writes gpurun_out/ctx_sweep.jsonl and a table
# gpurun_out/ctx_sweep.txt (KV bytes per step = 28 layers x 2 KV heads x 128
# x 2 (K, V) x 2 B = 28,672 B per cached position of the positive stream).
# usage: tools/ctx_sweep.sh [steps] [contexts...]
set -u
steps="${1:-200}"; shift || true
ctxs="${*:-0 4096 16384 32768 65000}"
mkdir -p gpurun_out
out=gpurun_out/ctx_sweep.jsonl; : > "$out"
for c in $ctxs; do
  echo "[ctx_sweep] context $c"
  timeout -k 10 300 python bench.py --context "$c" --steps "$steps" --warmup 10 --no-cpu-baseline \
      > "gpurun_out/ctx_sweep_$c.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[ctx_sweep] context $c rc=$rc"; tail -5 "gpurun_out/ctx_sweep_$c.log"; exit $rc; fi
  grep '^{"metric"' "gpurun_out/ctx_sweep_$c.log" | tail -1 | python -c "import sys, json; d = json.loads(sys.stdin.read()); d['context'] = $c; print(json.dumps(d))" >> "$out"
done
python - "$out" <<'EOF' | tee gpurun_out/ctx_sweep.txt
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
# keys per step: the mean cached length over the timed steps (config.context_start .. context_end)
print(f"{'context':>8} {'keys':>7} {'ms/step':>8} {'frames/s':>9} {'audio-s/s':>9} {'KV GB/step':>10} {'KV TB/s':>8}")
for r in rows:
    ms = r["ms_per_step"]
    keys = (r["config"]["context_start"] + r["config"]["context_end"]) / 2
    kv = 28672 * keys / 1e9
    print(f"{r['context']:>8} {keys:>7.0f} {ms:>8.4f} {1e3 / ms:>9.1f} {r['value']:>9.2f} {kv:>10.3f} {kv / ms:>8.3f}")
EOF
