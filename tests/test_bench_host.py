"""bench.py's host-side pieces that need no GPU: the host core count and the reference CPU baseline
(oracle/_ref/ref_driver, the reference built from its sources by __graft_entry__.build()), on a
tiny frame: the faster of -t usable / -t nproc is the figure, and both runs are reported."""
import os
import sys

import pytest

from _util import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_host_cores_usable_is_the_smallest_limit():
    c = bench.host_cores()
    assert c["usable"] >= 1
    assert c["usable"] <= c["nproc"] and c["usable"] <= c["affinity"]
    if c["cgroup_quota"]:
        assert c["usable"] <= c["cgroup_quota"]


@pytest.mark.skipif(not os.path.exists(bench.REF_DRIVER), reason="oracle/_ref/ref_driver not built")
def test_reference_baseline_reports_both_thread_counts():
    dae = os.path.join(REPO, "scenes", "CBspheres.dae")
    cores = {"nproc": 2, "affinity": 2, "cgroup_quota": 1, "usable": 1}
    r = bench.cpu_baseline_reference(dae, "CBspheres", 32, 24, 3, threads=1, cores=cores, min_spp=4)
    assert r is not None and r["kind"] == "reference" and r["unit"] == "Msamples/s"
    tried = r["threads_tried"]
    assert set(tried) == {"1", "2"}
    best = max(tried, key=lambda t: tried[t]["value"])
    assert r["cores"] == int(best)
    assert abs(r["value"] - tried[best]["value"]) <= 1e-5 * max(1.0, r["value"])
    assert r["spp1"]["value"] > 0 and "-t 1 / -t 2" in r["sample"]
