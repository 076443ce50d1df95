"""Host half of the device path (string dictionaries -> bitsets, catalogue SoA, topology groups) under
AddressSanitizer on CPU: kp_solve_validate over every scenario family the GPU parity tests use. The
product's kernels are not involved (no device here); GPU sanitizers are not available on the pool."""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "karpenter-provider-aws_amd")

SCRIPT = r'''
import sys
sys.path.insert(0, %(pkg)r)
import kpamd
kpamd.load_lib(%(lib)r)
from kpamd import catalog, synth
cat = catalog.build_catalog(kpamd.load_lib())
for seed in range(16):
    assert kpamd.validate(synth.random_topology_problem(cat, seed, n_existing=[0, 12, 30][seed %% 3])) == 0, seed
assert kpamd.validate(synth.config3(cat, n_pods=2000, n_deployments=40, n_existing=100)) == 0
for seed in range(12):
    assert kpamd.validate(synth.random_problem(cat, seed, n_types=150, n_pods=250, n_pools=3,
                                               n_existing=[0, 5, 40][seed %% 3], n_shapes=20)) == 0
assert kpamd.validate(synth.config2(cat, n_pods=2000)) == 0
assert kpamd.validate(synth.config5(cat, n_pods=4000)) == 0
sys.path.insert(0, %(tests)r)
import test_hostports_volumes as hp, test_pod_antiaffinity as pa  # ABI v6 families: ports, volumes, pod terms
for seed in range(4):
    assert kpamd.validate(hp.add_ports_and_volumes(synth.random_problem(cat, seed, n_types=120, n_pods=200, n_pools=3,
                                                                       n_existing=8, n_shapes=16), seed)) == 0
    assert kpamd.validate(pa.add_anti(synth.random_problem(cat, 500 + seed, n_types=120, n_pods=200, n_pools=3,
                                                           n_existing=10, n_shapes=14), seed)) == 0
print("asan-ok")
'''


def test_host_compile_under_asan():
    lib = os.path.join(PKG, "build", "asan", "libkp.so")
    subprocess.check_call(["make", "-s", "-C", PKG, "asan"], stdout=subprocess.DEVNULL)
    rt = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    assert rt, "ASan runtime missing"
    env = dict(os.environ, LD_PRELOAD=rt[-1], ASAN_OPTIONS="detect_leaks=0")
    out = subprocess.run([sys.executable, "-c", SCRIPT % {"pkg": PKG, "lib": lib, "tests": os.path.join(REPO, "tests")}], env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0 and "asan-ok" in out.stdout, out.stderr[-3000:]
