"""Build an A/B variant of libtorj_hip.so from a patched copy of the sources
(profiling aid, never shipped): python scripts/mkvariant.py NAME [-DFLAG ...] 'file|||old|||new' ...
-> torj.jl_amd/build/variants/libtorj_hip_NAME.so (run by scripts/gpu_call.sh AB=... or scripts/gpu_ab.sh); -D... arguments are
extra compile flags (e.g. -DTORJ_WARM_PROF, the warm alpha's region timers: tools/warm_prof.py)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1]
flags = [a for a in sys.argv[2:] if a.startswith("-")]
specs = [a for a in sys.argv[2:] if not a.startswith("-")]
base = f"/tmp/torj_variant/{name}"
shutil.rmtree(base, ignore_errors=True)
shutil.copytree(os.path.join(ROOT, "torj.jl_amd", "csrc"), f"{base}/pkg/csrc")
shutil.copytree(os.path.join(ROOT, "include"), f"{base}/include")
for spec in specs:
    f, a, b = spec.split("|||")
    p = f"{base}/pkg/csrc/{f}"
    s = open(p).read()
    assert a in s, (f, a[:60])
    open(p, "w").write(s.replace(a, b))
out = os.path.join(ROOT, "torj.jl_amd", "build", "variants", f"libtorj_hip_{name}.so")
os.makedirs(os.path.dirname(out), exist_ok=True)
subprocess.check_call(["make", "-s", "-C", f"{base}/pkg/csrc", f"LIB={out}", "EXTRA=" + " ".join(flags)])
print(out)
