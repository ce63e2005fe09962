"""CPU-side checks of the C ABI: the library builds, loads, and exports every entry
point include/safelife_hip.h declares; the ctypes structs match the header layout."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "safelife_hip.h")


def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sl_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from safelife_amd import _lib
    _lib.build()
    return _lib.lib()


def test_exports_every_declared_symbol(lib):
    names = _declared_functions()
    assert len(names) >= 8
    for n in names:
        assert hasattr(lib, n), n
    nm = subprocess.check_output(["nm", "-D", "--defined-only",
                                  os.path.join(REPO, "safelife-k2_amd", "safelife_amd", "_native",
                                               "libsafelife_hip.so")]).decode()
    for n in names:
        assert re.search(r"\bT %s$" % n, nm, re.M), n


def test_version(lib):
    assert b"gfx950" in lib.sl_version()


def test_struct_layout_matches_header(tmp_path):
    """Compile a tiny C program with the header and compare offsets with ctypes."""
    from safelife_amd import _lib
    prog = tmp_path / "layout.c"
    fields = {"sl_env_state": _lib.EnvState, "sl_level_pool": _lib.LevelPool,
              "sl_env_cfg": _lib.EnvCfg, "sl_capture": _lib.Capture, "sl_mt19937": _lib.MT19937}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "%s"' % HEADER,
             'int main(void){']
    for cname, cls in fields.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in cls._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-o", str(exe), str(prog)])
    out = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)]).decode().split("\n")
               if l)
    for cname, cls in fields.items():
        assert int(out[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(out["%s.%s" % (cname, f)]) == getattr(cls, f).offset, (cname, f)


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from safelife_amd import speedups, _lib
    import numpy as np
    # numpy boards take the host engine; the device entries fail loudly
    assert speedups.advance_board(np.zeros((4, 4), np.uint16)).shape == (4, 4)
    with pytest.raises(_lib.HipUnavailable):
        speedups.advance_board(torch.zeros((4, 4), dtype=torch.uint16))
    with pytest.raises(_lib.HipUnavailable):
        speedups.advance_boards(torch.zeros((2, 4, 4), dtype=torch.uint16))
    from safelife_amd import SafeLifeEnv, SafeLifeVecEnv, LevelPool
    from safelife_amd.side_effects import side_effect_densities
    level = {"board": np.zeros((8, 8), np.uint16), "goals": np.zeros((8, 8), np.uint16)}
    with pytest.raises(_lib.HipUnavailable):
        SafeLifeEnv(iter([level])).reset()
    with pytest.raises(_lib.HipUnavailable):
        SafeLifeVecEnv(LevelPool.from_levels([level]), 4)
    with pytest.raises(_lib.HipUnavailable):
        side_effect_densities(np.zeros((1, 8, 8), np.uint16), np.zeros((1, 8, 8), np.uint16),
                              [0], 0.3, 2)
