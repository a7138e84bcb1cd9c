"""The C-ABI library loads and exports every declared symbol (no compute: no GPU needed)."""
import ctypes
import os
import re

import pytest

from conftest import PKG_NAME, REPO


def _declared():
    src = open(os.path.join(REPO, "include", "openpose_hip.h")).read()
    return sorted(set(re.findall(r"\b(op_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported(lib):
    L = ctypes.CDLL(lib.LIB_PATH)
    decl = _declared()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(lib.EXPORTED) == decl


def test_loaded_library_is_built_from_this_tree(lib):
    """op_build_info reports the digest of the sources the loaded .so was
    compiled from (csrc/Makefile bakes it in); it must equal the digest of the checked-out csrc/ and
    include/ -- a stale or foreign binary fails here (and in smoke() on the GPU box)."""
    got = lib.build_info()
    assert re.fullmatch(r"sha256:[0-9a-f]{64};defs=.*", got), got
    # advisor r05: the build flags are part of the provenance; the product library has none
    assert lib.build_flags() == "", "experiment build flags in the product library: %r" % lib.build_flags()
    assert lib.build_digest() == lib.source_digest(), "libopenpose_hip.so was not built from this tree's sources: rebuild it"
    assert lib.check_provenance() == lib.build_digest()
    buf = ctypes.create_string_buffer(8)
    assert lib.lib().op_build_info(buf, len(buf)) == lib.OP_ERR_INVALID  # too small: refused, nothing written


def test_provenance_without_sources(lib, monkeypatch):
    """advisor r05: with no csrc/ to hash (an install without sources) the digest is unverifiable:
    check_provenance() reports None instead of failing on a mismatch."""
    monkeypatch.setattr(lib, "source_digest", lambda csrc=None: None)
    assert lib.check_provenance() is None


def test_build_flags_reach_the_provenance(tmp_path):
    """advisor r05: an experiment build's flags (DEFS) are baked into op_build_info, so a probe
    library copied over the product one fails check_provenance(); build_info.cpp alone, compiled the
    way the Makefile compiles it."""
    import subprocess
    src = os.path.join(REPO, PKG_NAME, "csrc", "build_info.cpp")
    so = str(tmp_path / "bi.so")
    subprocess.run(["g++", "-shared", "-fPIC", "-std=c++17", "-I", os.path.join(REPO, "include"),
                    "-DOP_BUILD_DIGEST=\"%s\"" % ("0" * 64), "-DOP_BUILD_FLAGS=\"-DC1P_PROBE_NO11=1\"",
                    src, "-o", so], check=True)
    L = ctypes.CDLL(so)
    buf = ctypes.create_string_buffer(256)
    assert L.op_build_info(buf, len(buf)) == 0
    assert buf.value.decode() == "sha256:" + "0" * 64 + ";defs=-DC1P_PROBE_NO11=1"


def test_layer_table_matches_cocoposenet(lib):
    from oracle.forward import LAYERS
    assert lib.layer_table() == LAYERS


def test_forward_flops(lib):
    # 271.9 GFLOP per 368x368 frame, 484.6 at 656x368
    assert abs(lib.forward_flops(368, 368) / 1e9 - 271.868) < 0.01
    assert abs(lib.forward_flops(368, 656) / 1e9 - 484.6) < 0.1


def test_default_params_mirror_entity(lib, pkg):
    p = lib.default_params()
    prm = pkg.params
    assert p.inference_img_size == prm["inference_img_size"] and p.heatmap_size == prm["heatmap_size"]
    assert p.gaussian_sigma == prm["gaussian_sigma"] and p.n_integ_points == prm["n_integ_points"]
    assert [[p.limbs_point[i][0], p.limbs_point[i][1]] for i in range(19)] == [[int(a), int(b)] for a, b in prm["limbs_point"]]


def test_no_silent_cpu_path(lib):
    """Without a GPU the product path must fail loudly, never fall back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        lib.Context(0)


def test_library_resolves_its_own_symbols():
    """Every op:: symbol the library uses is defined in it (a shared library links with undefined
    symbols; they would only fail at load time on the GPU box)."""
    import subprocess
    so = os.path.join(REPO, PKG_NAME, "libopenpose_hip.so")
    out = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True, check=True).stdout
    own = [l for l in out.splitlines() if "_ZN2op" in l or " op_" in l]
    assert not own, own


@pytest.mark.parametrize("preset", [None, "4", "16"])
def test_loader_leaves_the_environment_alone(preset):
    """Loading the library does not rewrite the host process's environment (round 3: the
    GPU_MAX_HW_QUEUES raise went with the detect_precise side stream)."""
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("GPU_MAX_HW_QUEUES", None)
    if preset is not None:
        env["GPU_MAX_HW_QUEUES"] = preset
    code = ("import importlib, os, sys; sys.path.insert(0, %r); before = dict(os.environ); "
            "m = importlib.import_module(%r + '._lib'); m.lib(); print(before == dict(os.environ), "
            "os.environ.get('GPU_MAX_HW_QUEUES'))" % (REPO, PKG_NAME))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "True %s" % preset


def test_census_and_profile_slots_mirror_the_header(lib):
    """_lib.CENSUS / CENSUS_SLOTS / PROFILE_CLASSES name exactly the header's OP_CENSUS_* and
    OP_PROFILE_CLASSES slots (the census and profile readers index C arrays by them)."""
    src = open(os.path.join(REPO, "include", "openpose_hip.h")).read()
    defs = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+(OP_CENSUS_[A-Z0-9_]+)\s+(\d+)", src)}
    assert defs.pop("OP_CENSUS_SLOTS") == lib.CENSUS_SLOTS
    named = {k: v for k, v in defs.items()}
    assert sorted(lib.CENSUS.values()) == sorted(v for v in named.values() if v >= 11)
    for name, slot in lib.CENSUS.items():
        assert named["OP_CENSUS_" + name.upper()] == slot, name
    assert all(v < lib.CENSUS_SLOTS for v in named.values())
    m = re.search(r"#define\s+OP_PROFILE_CLASSES\s+(\d+)", src)
    assert int(m.group(1)) == len(lib.Context.PROFILE_CLASSES)
