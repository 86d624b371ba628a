#!/bin/bash
# The N = 2 same-device rehearsals (scripts/gpu_rehearsal_r06.sh) and a short
# default C3 line, printing the roofline traffic each found (the N >= 2 lines
# take device 0's per-launch bytes from the single-device profile of the same
# build; placement switches do not enter the match) -> gpurun_out/reh/
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_rehearsal_r06.sh || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-exact --no-host-api --steps 3 > gpurun_out/reh/c3.log 2>&1 || { tail -20 gpurun_out/reh/c3.log; exit 1; }
grep '^{' gpurun_out/reh/c3.log > gpurun_out/reh/c3.json
python - <<'PY'
import json
for f in ("reh/bench_torchrun2_same_device_rehearsal.json", "reh/bench_lib2_same_device_rehearsal.json", "reh/c3.json"):
    d = json.load(open("gpurun_out/" + f))
    print(f, d["value"], d["roofline"].get("traffic"), d["roofline"].get("traffic_source"))
PY
