"""The C-ABI's multi-GPU frame reduce on hardware (bdpt_reduce_*, ABI v9): RCCL's
ncclReduce of the contexts' eye and light frames into the root context's, plus the on-device sum of
contexts that share a GPU (RCCL refuses two ranks on one device, so a one-GPU box exercises both
halves: every context on device 0 = a one-rank communicator after the device-side sum).

The reduced frame must equal one render of all the samples (the RNG is keyed by the global sample
index; only the fp32 summation order differs), the other contexts' frames must be unchanged, and
under the PathTracer the reduced sampleCountBuffer must be the whole frame's."""
import numpy as np
import pytest

import bdpt_amd as B
from _util import device_count, golden_scene

pytestmark = pytest.mark.gpu

W, H, M = 96, 72, 5


def _render(sc, spp, begin, count, **kw):
    pt = B.BidirectionalPathTracer(sc, W, H, spp, M, seed=5489, **kw)
    pt.raytrace_tiles([], begin, count)
    return pt


def test_one_context_one_rank_is_identity():
    """-g 1: one context, a one-rank communicator; the in-place reduce leaves the frame bit-equal."""
    sc = golden_scene("CBspheres", W, H)
    pt = _render(sc, 4, 0, 4)
    before = pt.read_frame(B.FRAME_SAMPLE)
    red = B.FrameReducer([pt])
    assert red.ranks == 1
    red.reduce(0)
    after = pt.read_frame(B.FRAME_SAMPLE)
    red.close()
    pt.close()
    assert np.array_equal(before, after)


@pytest.mark.parametrize("nctx,root", [(2, 0), (3, 2)])
def test_contexts_on_one_device_reduce_to_single_render(nctx, root):
    sc = golden_scene("CBgems", W, H)
    SPP = 6
    pts = [_render(sc, SPP, SPP * k // nctx, SPP * (k + 1) // nctx - SPP * k // nctx) for k in range(nctx)]
    own = [p.read_frame(B.FRAME_SAMPLE) for p in pts]
    eye = [p.read_frame(B.FRAME_EYE) for p in pts]
    red = B.FrameReducer(pts)
    assert red.ranks == 1   # every context on device 0: one RCCL rank after the on-device sum
    red.reduce(root)
    got = pts[root].read_frame(B.FRAME_SAMPLE).astype(np.float64)
    got_eye = pts[root].read_frame(B.FRAME_EYE).astype(np.float64)
    for k, p in enumerate(pts):   # the non-root frames are untouched
        if k != root:
            assert np.array_equal(p.read_frame(B.FRAME_SAMPLE), own[k])
    red.close()
    for p in pts:
        p.close()
    single = _render(sc, SPP, 0, SPP)
    ref = single.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    ref_eye = single.read_frame(B.FRAME_EYE).astype(np.float64)
    single.close()
    rmse = float(np.sqrt(np.mean((got - ref) ** 2)))
    print(f"{nctx} contexts -> root {root}: rmse vs single render {rmse:.3e}")
    assert rmse < 1e-6
    assert np.allclose(got_eye, ref_eye, atol=1e-5)     # the eye and light frames are reduced separately
    assert np.allclose(got_eye, np.sum(eye, axis=0), atol=1e-6)


def test_reduce_twice_after_clear_and_rerender():
    """The reducer persists across steps (the communicator is made once): clear, render the next
    sample range, reduce again — the root then holds only the new step's sum."""
    sc = golden_scene("CBspheres", W, H)
    pts = [_render(sc, 4, 2 * k, 2) for k in range(2)]
    red = B.FrameReducer(pts)
    red.reduce(0)
    for k, p in enumerate(pts):
        p.clear()
        p.raytrace_tiles([], 4 + 2 * k, 2)
    red.reduce(0)
    got = pts[0].read_frame(B.FRAME_SAMPLE).astype(np.float64)
    red.close()
    for p in pts:
        p.close()
    single = _render(sc, 4, 4, 4)
    ref = single.read_frame(B.FRAME_SAMPLE).astype(np.float64)
    single.close()
    assert float(np.sqrt(np.mean((got - ref) ** 2))) < 1e-6


def test_pathtracer_row_bands_reduce_frames_and_counts():
    """The PathTracer splits whole pixels by row bands; the reduce sums its frames and its
    sampleCountBuffer (int32), so the root holds the whole image and every pixel's count."""
    sc = golden_scene("CBspheres", W, H)
    SPP = 4
    bands = [(0, 0, W, H // 2), (0, H // 2, W, H - H // 2)]
    pts = []
    for b in bands:
        p = B.PathTracer(sc, W, H, SPP, M, seed=5489, max_tolerance=0.0)
        p.raytrace_tiles([b], 0, SPP)
        pts.append(p)
    red = B.FrameReducer(pts)
    red.reduce(0)
    got = pts[0].read_frame(B.FRAME_SAMPLE)
    counts = pts[0].read_sample_counts()
    red.close()
    for p in pts:
        p.close()
    whole = B.PathTracer(sc, W, H, SPP, M, seed=5489, max_tolerance=0.0)
    whole.raytrace_tiles([], 0, SPP)
    ref = whole.read_frame(B.FRAME_SAMPLE)
    ref_counts = whole.read_sample_counts()
    whole.close()
    # the reference runs whole batches (pathtracer.cpp:301-337): ns_aa 4 with samplesPerBatch 32 and
    # no early stop records num_samples = 32 for every pixel
    assert np.array_equal(counts, ref_counts) and (counts == 32).all()
    assert np.array_equal(got, ref)   # disjoint bands: each pixel sums one value and zeros


# --- >= 2 devices: run by themselves on the first multi-GPU box; skipped with the reason here ----

@pytest.mark.skipif(device_count() < 2, reason="needs >= 2 visible GPUs (this pool's boxes have one): "
                                               "the two-rank ncclReduce between distinct devices")
@pytest.mark.parametrize("root", [0, 1, 2])
def test_contexts_on_two_devices_reduce_to_single_render(root):
    """Three contexts over devices 0, 1, 0: two RCCL ranks (device 0's pair summed on it first),
    the cross-device grouped ncclReduce into the root's frames with the root on either device; the
    reduced frame equals one render of all the samples and the non-root frames are untouched."""
    sc = golden_scene("CBgems", W, H)
    SPP, devs = 6, [0, 1, 0]
    pts = [_render(sc, SPP, 2 * k, 2, device=d) for k, d in enumerate(devs)]
    own = [p.read_frame(B.FRAME_SAMPLE) for p in pts]
    red = B.FrameReducer(pts)
    assert red.ranks == 2
    red.reduce(root)
    got = pts[root].read_frame(B.FRAME_SAMPLE).astype(np.float64)
    for k, p in enumerate(pts):
        if k != root:
            assert np.array_equal(p.read_frame(B.FRAME_SAMPLE), own[k])
    # a second step through the same communicator: clear, render the next ranges, reduce again
    for k, p in enumerate(pts):
        p.clear()
        p.raytrace_tiles([], SPP + 2 * k, 2)
    red.reduce(root)
    got2 = pts[root].read_frame(B.FRAME_SAMPLE).astype(np.float64)
    red.close()
    for p in pts:
        p.close()
    for lo, g in ((0, got), (SPP, got2)):
        single = _render(sc, SPP, lo, SPP)
        ref = single.read_frame(B.FRAME_SAMPLE).astype(np.float64)
        single.close()
        assert float(np.sqrt(np.mean((g - ref) ** 2))) < 1e-6


def test_renderer_close_closes_its_reducer_first():
    """Closing a renderer before its reducer (or interpreter-exit finaliser order) must not leave
    the reducer pointing at a freed context: the renderer closes its reducers first."""
    sc = golden_scene("CBspheres", W, H)
    pts = [_render(sc, 4, 2 * k, 2) for k in range(2)]
    red = B.FrameReducer(pts)
    red.reduce(0)
    pts[1].close()                 # before red.close()
    assert red.h is None
    with pytest.raises(B.BDPTError):
        red.reduce(0)
    red.close()                    # idempotent
    pts[0].close()
    with pytest.raises(B.BDPTError):
        B.FrameReducer(pts)        # closed renderers are refused
