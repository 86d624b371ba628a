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
