"""The C-ABI shared library: loads, exports every entry point of include/pbn_env.h,
and rejects bad descriptors / arguments before touching the device (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import pytest

from pbn_rl_amd import _lib
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec, PbnNetDesc

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "pbn_env.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(pbn_\w+)\s*\(", text, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.load()


def test_header_declares_the_abi():
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (\w+)$", out, re.M))
    for name in declared_functions():
        assert name in exported, name
        assert hasattr(lib, name)


def test_abi_version(lib):
    assert lib.pbn_abi_version() == 11


def test_descriptor_layout_matches_header(tmp_path):
    """ctypes' pbn_net_desc == the C compiler's (sizeof and every offsetof, from the header)."""
    import subprocess
    fields = [f for f, _ in PbnNetDesc._fields_]
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "pbn_env.h"\nint main(void) {\n'
                   '  printf("%zu\\n", sizeof(pbn_net_desc));\n' +
                   "".join(f'  printf("%zu\\n", offsetof(pbn_net_desc, {f}));\n' for f in fields) + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    inc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "include")
    subprocess.run(["gcc", "-I", inc, "-o", str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got[0] == ctypes.sizeof(PbnNetDesc)
    assert got[1:] == [getattr(PbnNetDesc, f).offset for f in fields]


def _create(lib, spec):
    h = ctypes.c_void_p()
    rc = lib.pbn_net_create(ctypes.addressof(spec.desc), ctypes.byref(h))
    return rc, lib.pbn_last_error().decode()


@pytest.mark.parametrize("field,value,msg", [
    ("prob_bits", 5, "prob_bits"),
    ("horizon", 300, "horizon"),
    ("settle_max", 5000, "settle_max"),
    ("n_nodes", 0, "n_nodes"),
    ("n_attractors", 255, "n_attractors"),
])
def test_create_rejects_bad_descriptor(lib, field, value, msg):
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    setattr(spec.desc, field, value)
    rc, err = _create(lib, spec)
    assert rc == -22 and msg in err


def test_create_rejects_bad_thresholds(lib):
    spec = EnvSpec(load_network("pbn7"), load_attractors("pbn7"))
    last = spec.arrays["node_func_start"][1] - 1
    spec.arrays["func_threshold"][last] = 1  # last threshold of node 0 must be 2^prob_bits
    rc, err = _create(lib, spec)
    assert rc == -22 and "threshold" in err


def test_step_rejects_null_net(lib):
    rc = lib.pbn_step(None, 0, 0, 0, 32, 3, None, None, None, None, None, None, None, None, None)
    assert rc == -22
    assert lib.pbn_reset(None, 0, 0, 0, 32, None, None, None, None) == -22
