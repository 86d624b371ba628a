"""bench.py's --gpus handling on CPU (no device work happens before these
checks): too few visible devices, a WORLD_SIZE that disagrees with --gpus and
--gpus < 1 all exit non-zero with a message instead of measuring something else."""
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("TORJ_BEAM_SAME_DEVICE", None)
    env["HIP_VISIBLE_DEVICES"] = ""  # hide any device (the CPU suite may run anywhere)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_gpus_more_than_visible_fails_loudly():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "--gpus 2 needs 2 visible HIP devices, found 0" in r.stderr
    assert r.stdout.strip() == ""  # no bench line


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4"], {"WORLD_SIZE": "2"})
    assert r.returncode != 0 and "WORLD_SIZE = 2" in r.stderr


def test_gpus_below_one_rejected():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus 0" in r.stderr
