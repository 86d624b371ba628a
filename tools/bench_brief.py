"""One-line summary of a bench.py log: value, trace-kernel ms, roofline fraction."""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        r = d["roofline"]
        frac = r["frac"] if r["frac"] is not None else float("nan")
        print(f"{d['config']['workload'][:2]} value {d['value']:.4e} ray-steps/s  "
              f"kernel {r['kernel_ms']:.1f} ms  post {r['deposition_kernels_ms']:.1f} ms  frac {frac:.3f}")
