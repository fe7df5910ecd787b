"""CPU: the C-ABI library builds, loads without a GPU and exports every function the
header declares."""
import os
import re
import subprocess

from conftest import REPO


def _header_functions():
    src = open(os.path.join(REPO, 'include', 'acinoset_hip.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(acs_[a-z0-9_]+)\s*\(', src)))


def test_library_loads_and_exports_header_symbols():
    from acinoset_amd import _native
    lib = _native.load_library()
    assert lib.acs_abi_version() == _native.ABI_VERSION == 5
    nm = subprocess.run(['nm', '-D', '--defined-only', _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r'\b(acs_[a-z0-9_]+)\b', nm))
    missing = [f for f in _header_functions() if f not in exported]
    assert not missing, missing
    for f in _header_functions():
        assert hasattr(lib, f)


def test_no_gpu_means_loud_failure_not_fallback():
    """Creating a context without a gfx950 device must raise, never silently compute."""
    import pytest
    from acinoset_amd import _native
    n = _native.C.c_int(-1)
    _native.load_library().acs_device_count(_native.C.byref(n))
    if n.value > 0:
        pytest.skip('a GPU is visible')
    with pytest.raises(_native.NativeUnavailable):
        _native.Context(0)


def test_kernels_are_gfx950_code_objects():
    from acinoset_amd import _native
    data = open(_native.LIB_PATH, 'rb').read()
    assert b'amdgcn-amd-amdhsa--gfx950' in data


def test_alloc_counter_needs_no_gpu():
    """acs_alloc_events (the allocation counter the bench's timed multi-GPU region is checked
    with) is callable without a device and never decreases."""
    from acinoset_amd import _native
    a = _native.alloc_events()
    assert a >= 0 and _native.alloc_events() >= a
