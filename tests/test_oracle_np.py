"""The NumPy / SciPy restatement bench.py's cpu_baseline times (oracle/postproc_np.py) against the
reference's own outputs (tests/golden/, made by make_golden.py) and the C restatement: it must be
the reference's post-process, not merely cost like it."""
import numpy as np
import pytest

from conftest import golden_cases, load_golden
from oracle import postproc as P
from oracle import postproc_np as N

# the large cases take seconds in the per-pair Python loops: keep the CPU suite short
FAST = [c for c in golden_cases() if c not in ("noise_crowd", "twenty_720p")]


@pytest.mark.parametrize("case", FAST)
def test_numpy_postprocess_matches_reference(case):
    d = load_golden(case)
    mh, mw = int(d["map_h"]), int(d["map_w"])
    heat = N.resize_align_corners(d["heat_low"], mh, mw)
    assert np.array_equal(heat, P.resize_images(d["heat_low"], mh, mw))
    peaks = N.find_peaks(heat)
    assert np.array_equal(np.asarray(peaks).reshape(-1, 5), d["all_peaks"])
    if int(d["status"]) == 1:
        poses, scores = N.postprocess(d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
        assert poses.shape == (0, 18, 3) and scores.shape == (0,)
        return
    pafs = N.resize_align_corners(d["paf_low"], mh, mw)
    conns = N.connect_limbs(pafs, peaks, mw)
    assert np.array_equal(np.concatenate(conns), d["conn"])
    if int(d["status"]) == 4:
        with pytest.raises(IndexError):
            N.group_people(conns, peaks)
        return
    assert np.array_equal(N.group_people(conns, peaks), d["subsets"])
    poses, scores = N.postprocess(d["paf_low"], d["heat_low"], int(d["orig_h"]), int(d["orig_w"]))
    assert np.array_equal(np.asarray(poses, np.float64).reshape(d["poses"].shape), d["poses"])
    assert np.array_equal(scores, d["scores"])


def test_numpy_grouping_indexerror_like_reference():
    d = load_golden("grouping_indexerror")
    off = d["conn_off"]
    conns = [d["conn"][off[l]:off[l + 1]] for l in range(19)]
    with pytest.raises(IndexError):
        N.group_people(conns, d["all_peaks"])


def test_numpy_resize_matches_c_restatement_odd_sizes():
    x = np.random.default_rng(4).standard_normal((3, 17, 29)).astype(np.float32)
    for oh, ow in ((61, 45), (17, 29), (5, 90)):
        assert np.array_equal(N.resize_align_corners(x, oh, ow), P.resize_images(x, oh, ow))
