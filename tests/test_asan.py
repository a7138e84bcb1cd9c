"""Host-side AddressSanitizer run of the C ABI (SURVEY §5 "race detection / sanitizers"): the
library's host code built with -fsanitize=address (csrc/Makefile `asan`, host code only) is
loaded into a child Python with the ASan runtime preloaded, and every entry point that runs
without a GPU is driven -- tables, parameter defaults, FLOP counts, argument validation and the
error paths of the device entry points (no device here: they must fail cleanly, not touch
memory they do not own).  Any ASan report aborts the child and fails the test."""
import os
import subprocess
import sys

import pytest

from conftest import REPO, PKG_NAME

CSRC = os.path.join(REPO, PKG_NAME, "csrc")
ASAN_RT = "/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so"

CHILD = r'''
import ctypes, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from importlib import import_module
L = import_module("chainer_realtime_multi-person_pose_estimation_amd._lib")
F = import_module("chainer_realtime_multi-person_pose_estimation_amd.frames")
lib = L.lib()
assert lib._name.endswith("libopenpose_hip.asan.so"), lib._name
assert L.build_digest() == L.source_digest()
p = L.OpParams(); assert lib.op_default_params(ctypes.byref(p)) == 0
lim = L.OpLimits(); assert lib.op_default_limits(ctypes.byref(lim)) == 0
assert lib.op_default_params(None) != 0 and lib.op_default_limits(None) != 0
t = L.layer_table(); assert len(t) == 92 and t[0][1:] == (3, 64, 3)
for arch in ("facenet", "handnet"):
    assert len(L.cpm_layer_table(arch)) > 0
assert lib.op_layer_info(92, None, None, None, None) != 0 and lib.op_layer_info(-1, None, None, None, None) != 0
assert abs(L.forward_flops(368, 368) - 271.87e9) < 0.01e9
# device entry points without a device / with bad arguments: clean errors
h = ctypes.c_void_p()
rc = lib.op_create(ctypes.byref(p), ctypes.byref(lim), 0, ctypes.byref(h))
assert rc != 0 and not h.value and len(L.last_error()) > 0
for fn, args in [("op_destroy", (None,)), ("op_cpm_destroy", (None,)), ("op_comm_destroy", (None,)),
                 ("op_host_free", (None,)), ("op_train_destroy", (None,))]:
    assert getattr(lib, fn)(*args) == 0, fn
assert lib.op_detect(None, None, 0, 0, 0, None, None, 0, None) != 0
assert lib.op_fetch_maps(None, 0, 1, None, None, None, None) != 0
assert lib.op_upload_frames(None, None, 1, 8, 8) != 0
assert lib.op_pack_results(None, 0, 1, 4, 0, 1, None) != 0
assert lib.op_comm_gather_results(None, None, 0, 1, 4, 0, 1) != 0
assert lib.op_comm_wait(None, 1.0, None, None, None) != 0
assert lib.op_comm_create(None, 2, 0, None, 1.0, None) != 0
assert lib.op_stage_frames(None, None, 1, 8, 8) != 0 and lib.op_run_staged(None) != 0
assert lib.op_cpm_create(7, 0, ctypes.byref(h)) != 0 and lib.op_cpm_layer_count(7) <= 0
# host-side record format round trip
poses = np.arange(2 * 18 * 3, dtype=np.float64).reshape(2, 18, 3)
rec = F.pack_records([(3, 0, 9, poses, np.array([1.0, 2.0]))], 4)
assert F.unpack_records(rec, 4)[0][0] == 3
print("asan ok")
'''


@pytest.mark.skipif(not os.path.exists(ASAN_RT), reason="clang ASan runtime not in this image")
def test_c_abi_host_code_under_asan():
    subprocess.check_call(["make", "-s", "-j8", "-C", CSRC, "asan"])
    env = dict(os.environ, OP_LIB_VARIANT="asan", LD_PRELOAD=ASAN_RT,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:allocator_may_return_null=1",
               HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "asan ok" in p.stdout, (p.returncode, p.stdout[-3000:], p.stderr[-6000:])
    assert "AddressSanitizer" not in p.stderr, p.stderr[-6000:]
