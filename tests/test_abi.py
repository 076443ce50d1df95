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
    assert lib.kp_abi_version() == 12
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
    assert C.sizeof(abi.LaunchResult) == 12 * 4
    assert C.sizeof(abi.LaunchRequest) == C.sizeof(abi.Requirements) + C.sizeof(abi.ResourceList) + 8 + 8


def test_struct_sizes_match_the_c_header(tmp_path):
    """ctypes mirrors of the ABI structs have the sizes gcc gives the header's structs (ABI v6 host ports, volumes)."""
    import shutil
    import subprocess
    from kpamd import abi
    import pytest
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    pairs = {"kp_pod_shape": abi.PodShape, "kp_existing_node": abi.ExistingNode, "kp_host_port": abi.HostPort,
             "kp_cluster_node": abi.ClusterNode, "kp_solve_in": abi.SolveIn, "kp_topology_spread": abi.TopologySpread,
             "kp_nodepool": abi.NodePool, "kp_cluster": abi.Cluster,
             "kp_pod_affinity_term": abi.PodAffinityTerm, "kp_bound_pod": abi.BoundPod,
             "kp_offering": abi.Offering, "kp_offering_update": abi.OfferingUpdate, "kp_launch_result": abi.LaunchResult,
             "kp_solve_stats": abi.SolveStats, "kp_nodeclass": abi.NodeClass, "kp_kubelet": abi.Kubelet,
             "kp_eviction_value": abi.EvictionValue, "kp_choice": abi.Choice, "kp_sim_result": abi.SimResult,
             "kp_options": abi.Options, "kp_ec2_info": abi.EC2Info, "kp_nodeclaim_info": abi.NodeClaimInfo,
             "kp_launch_request": abi.LaunchRequest, "kp_feasibility_query": abi.FeasibilityQuery,
             "kp_instance_type": abi.InstanceType, "kp_preferred_term": abi.PreferredTerm,
             "kp_label_selector": abi.LabelSelector, "kp_pod": abi.Pod, "kp_overrides": abi.Overrides}
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "kp/kp_abi.h"\nint main(void){\n' +
                   "".join(f'printf("%zu\\n", sizeof({k}));\n' for k in pairs) + "return 0;}\n")
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.dirname(os.path.dirname(HDR)), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [C.sizeof(t) for t in pairs.values()], dict(zip(pairs, got))


def test_library_reads_no_environment():
    """ABI v12: no environment variable picks a kernel or a path in production (kp_overrides, set per context, replaces
    the test hooks): libkp.so does not import getenv / secure_getenv."""
    import shutil
    import subprocess
    import pytest
    if not shutil.which("nm"):
        pytest.skip("nm not available")
    syms = subprocess.check_output(["nm", "-D", "--undefined-only", kpamd.LIB_PATH], text=True)
    assert not [l for l in syms.splitlines() if l.split()[-1].split("@")[0] in ("getenv", "secure_getenv")]
