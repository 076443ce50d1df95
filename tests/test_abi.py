"""The C-ABI library loads and exports every symbol include/kp/kp_abi.h declares (no compute calls)."""
import ctypes as C
import os
import re

import kpamd

HDR = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "kp", "kp_abi.h")


def declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|uint32_t|uint64_t|void|const char\*)\s+(kp_\w+)\(", src, re.M)))


def test_all_declared_symbols_exported():
    lib = kpamd.load_lib()
    names = declared()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_struct_sizes():
    lib = kpamd.load_lib()
    assert lib.kp_abi_version() == 5
    from kpamd import abi
    assert C.sizeof(abi.ResourceList) == 12 * 8 + 8
    assert C.sizeof(abi.Offering) == 5 * 8 + 8 + 8


def test_no_device_is_an_error_not_a_fallback():
    """Without a HIP device kp_ctx_create must fail loudly (no CPU fallback exists)."""
    import torch
    if torch.cuda.is_available():
        return
    try:
        kpamd.Context(0)
    except kpamd.KPError as e:
        assert e.code == kpamd.abi.KP_E_DEVICE
    else:
        raise AssertionError("kp_ctx_create succeeded without a device")


def test_launch_struct_layouts():
    from kpamd import abi
    assert C.sizeof(abi.LaunchResult) == 10 * 4
    assert C.sizeof(abi.LaunchRequest) == C.sizeof(abi.Requirements) + C.sizeof(abi.ResourceList) + 8 + 8
