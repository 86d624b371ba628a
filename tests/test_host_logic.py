"""Host-side logic of the product on CPU: the ctypes mirror of torj_trace_cfg
against the C header's layout, argument mapping of the Python mirror, and the
argument validation the C ABI does before touching a device."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def test_trace_cfg_layout_matches_header(T, tmp_path):
    """torj_trace_cfg offsets and size from the C compiler == the ctypes mirror."""
    from torj_hip._lib import TraceCfg

    fields = [f for f, _ in TraceCfg._fields_]
    src = tmp_path / "cfg.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "torj_hip.h"\nint main(void) {\n'
                   + "".join(f'    printf("%zu\\n", offsetof(torj_trace_cfg, {f}));\n' for f in fields)
                   + '    printf("%zu\\n", sizeof(torj_trace_cfg));\n    return 0;\n}\n')
    exe = tmp_path / "cfg"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    want = [getattr(TraceCfg, f).offset for f in fields] + [ctypes.sizeof(TraceCfg)]
    assert got == want


def test_absorption_argument_mapping():
    from torj_hip.solve import ABSORPTION, _absorption_code

    assert _absorption_code(True) == 1 and _absorption_code(False) == 0
    assert _absorption_code(np.bool_(True)) == 1
    for name, code in ABSORPTION.items():
        assert _absorption_code(name) == code
        assert _absorption_code(code) == code
    with pytest.raises(ValueError):
        _absorption_code(4)
    with pytest.raises(KeyError):
        _absorption_code("warm")


def test_alpha_warm_validates_before_the_device(T):
    """iwarm and mode are checked before any device work (the error names them)."""
    with pytest.raises(T.TorjError, match="iwarm"):
        T.alpha_warm(6e11, 0.3, 0.5, 0.9, 0.1, 2000.0, 1.0, mode=1, iwarm=2)
    with pytest.raises(T.TorjError, match="mode"):
        T.alpha_warm(6e11, 0.3, 0.5, 0.9, 0.1, 2000.0, 1.0, mode=0, iwarm=1)


def test_beam_shard_layout_matches_header(T, tmp_path):
    """torj_beam_shard offsets and size from the C compiler == the ctypes mirror."""
    from torj_hip._lib import BeamShard

    fields = [f for f, _ in BeamShard._fields_]
    src = tmp_path / "shard.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "torj_hip.h"\nint main(void) {\n'
                   + "".join(f'    printf("%zu\\n", offsetof(torj_beam_shard, {f}));\n' for f in fields)
                   + '    printf("%zu\\n", sizeof(torj_beam_shard));\n    return 0;\n}\n')
    exe = tmp_path / "shard"
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    want = [getattr(BeamShard, f).offset for f in fields] + [ctypes.sizeof(BeamShard)]
    assert got == want


def test_make_beam_adaptive_stride_rejected_before_tracing(T):
    """integrator='adaptive' with traj_stride > 1 fails before any device work
    (the adaptive final state is no saved sample): no plasma handle is touched."""
    with pytest.raises(ValueError, match="adaptive"):
        T.make_beam(None, 2.5, 0.0, 0.4, 0.0, 0.5, 0.0174, 0.25, 92.5e9, 1, 0.2,
                    np.linspace(0, 1, 10), integrator="adaptive", traj_stride=2)


def test_fma_single_rounding():
    """solve.fma: a * b + c with one rounding (the kernel's v_fma_f64 of the
    final arc length), not the two of a * b + c."""
    from torj_hip.solve import fma

    a, b = 1.0 + 2.0 ** -30, 1.0 - 2.0 ** -30  # a b = 1 - 2^-60 exactly
    assert a * b - 1.0 == 0.0 and fma(a, b, -1.0) == -(2.0 ** -60)
    rng = np.random.default_rng(5)
    for s0, k, ds in zip(rng.uniform(0.1, 2.0, 200), rng.integers(1, 2001, 200), rng.uniform(1e-5, 1e-3, 200)):
        from fractions import Fraction

        assert fma(float(k), ds, s0) == float(Fraction(int(k)) * Fraction(ds) + Fraction(s0))


def test_group_shard_covers_the_beam_on_64_ray_groups():
    """parallel.group_shard (the bench's device shards) == torj_trace_beam's cut:
    contiguous, disjoint, covering, boundaries on 64-ray multiples."""
    from torj_hip.parallel import group_shard

    for n in (1, 63, 64, 65, 1038, 100203, 1005293):
        for S in (1, 2, 3, 8, 17):
            sl = [group_shard(n, S, k) for k in range(S)]
            assert sl[0].start == 0 and sl[-1].stop == n
            for a, b in zip(sl, sl[1:]):
                assert a.stop == b.start and a.stop % 64 == 0
    with pytest.raises(ValueError):
        group_shard(10, 2, 2)
