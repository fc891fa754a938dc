"""Parity statistics shared by the tests and bench.py's parity leg (test infrastructure).

Two comparisons that the GPU-vs-oracle-mode-2 RMSE alone does not make:

* fp64_agreement — the device's fp32 path (GPU, or oracle mode 2 which restates it) against
  oracle mode 1, the reference's fp64 arithmetic (CGL/include/CGL/vector3D.h:32-50) driven by
  the same counter RNG. Same seed, same samples, so the frames differ only where fp32 rounding
  flips a discrete decision of the walk: a visibility test at a connection ray's end
  (bidirection.cpp:418-433), the glass coin flip (advanced_bsdf.cpp:225), the `|contrib| > EPS_F`
  gate (:445), the area light's plane test (light.cpp:257-262), an edge hit. A flipped sample
  takes another path; every other sample agrees to fp32 rounding.
* null_calibrated_tails — the device's distribution against the reference's own mt19937 stream
  at the same spp, per pixel: the reference frame's deviations from a counter-RNG frame, in units
  of the per-pixel standard error, must have the same tail shares as those of independent
  counter-RNG frames (the "null"). The per-pixel values are heavy-tailed (caustic light-image
  splats), so the tails are compared against the null rather than against a Gaussian.
"""
import numpy as np

# a sample whose eye value moves by more than this, relative to |value| + 1e-2, took another path
DIVERGED_REL = 1e-3
AGREE_REL = 1e-5

# the fp32 tolerance vs the reference's fp64 arithmetic (README): measured on the
# five golden scenes, the Lucy stand-in and C5's shape (oracle mode 2 vs mode 1, 1-spp frames):
# diverged samples 0.4-2.8 %, RMSE / Monte Carlo noise 0.002-0.11
TOL_DIVERGED = 0.05        # at most 5 % of samples take another path
TOL_NOISE_RATIO = 0.25     # RMSE vs fp64 <= 0.25 x the per-pixel standard error, at any spp
TOL_AGREE = 0.95           # at least 95 % of samples agree with fp64 to 1e-5 relative


def fp64_agreement(eye32, samp32, eye64, samp64) -> dict:
    """eye32 / samp32 / eye64 / samp64: arrays (K, H, W, 3) of K single-sample frames (global sample
    indices 0..K-1, weight 1) of the fp32 path under test and of oracle mode 1. Returns the
    per-pixel RMSE of the K-spp images, the Monte Carlo noise of those images (per-pixel standard
    error from the spread of the 1-spp frames), their ratio, and the shares of samples (pixels of
    the 1-spp eye frames) that diverged / agree to AGREE_REL."""
    eye32, samp32, eye64, samp64 = (np.asarray(a, dtype=np.float64) for a in (eye32, samp32, eye64, samp64))
    K = samp32.shape[0]
    m32, m64 = samp32.mean(0), samp64.mean(0)
    rmse = float(np.sqrt(np.mean((m32 - m64) ** 2)))
    noise = float(np.sqrt(np.mean(samp64.var(0, ddof=1)) / K)) if K > 1 else float("nan")
    d = np.abs(eye32 - eye64).max(-1)
    scale = np.abs(eye64).max(-1) + 1e-2
    rel = d / scale
    return {"rmse_vs_fp64": rmse, "noise_rmse": noise, "rmse_over_noise": rmse / noise if noise > 0 else float("nan"),
            "diverged_frac": float(np.mean(rel > DIVERGED_REL)), "agree_1e-5_frac": float(np.mean(rel <= AGREE_REL)),
            "spp": K, "frame": f"{samp32.shape[2]}x{samp32.shape[1]}"}


def check_fp64_agreement(r: dict, what: str) -> None:
    assert r["diverged_frac"] <= TOL_DIVERGED, (what, r)
    assert r["rmse_over_noise"] <= TOL_NOISE_RATIO, (what, r)
    assert r["agree_1e-5_frac"] >= TOL_AGREE, (what, r)


TAIL_Z = (2.0, 3.0, 4.0, 6.0)
Z_CLIP = 4.0


def null_calibrated_tails(ref, A, nulls, var1, spp) -> dict:
    """ref: the reference's spp-sample frame; A: a counter-RNG frame of spp samples; nulls: further
    independent counter-RNG frames of spp samples; var1: per-pixel variance of a 1-spp
    counter-RNG frame (from frames independent of A and the nulls). z = (X - A) / sqrt(2 var1 /
    spp) per pixel and channel. Returns the tail shares P(|z| > t) over TAIL_Z and the clipped
    signed mean of z (a bias shows there first: 1 % of the image is ~0.15) for the reference and
    for each null frame."""
    se = np.sqrt(2.0 * var1 / spp)
    ok = se > 0

    def z(X):
        return (X - A)[ok] / se[ok]

    def tails(X):
        return np.array([np.mean(np.abs(z(X)) > t) for t in TAIL_Z])

    def cmean(X):
        return float(np.mean(np.clip(z(X), -Z_CLIP, Z_CLIP)))

    return {"ref_tails": tails(ref), "null_tails": np.array([tails(b) for b in nulls]),
            "ref_mean_z": cmean(ref), "null_mean_z": np.array([cmean(b) for b in nulls])}


def check_tails(r: dict, what: str) -> None:
    """The reference must sit inside the null's spread: each tail share at most the nulls' max
    (x1.25) plus 0.5 % of the pixels and at least half their mean minus 0.5 %; the clipped mean z
    within max(0.05, 3 sd of the nulls) of the nulls' mean."""
    tr, tn = r["ref_tails"], r["null_tails"]
    tn_mean, tn_max = tn.mean(0), tn.max(0)
    for k, t in enumerate(TAIL_Z):
        hi = max(tn_max[k] * 1.25, tn_mean[k] * 1.5) + 0.005
        lo = tn_mean[k] * 0.5 - 0.005
        assert lo <= tr[k] <= hi, (what, f"|z| > {t}: reference {tr[k]:.4f}, null mean {tn_mean[k]:.4f} "
                                         f"max {tn_max[k]:.4f}")
    nm = r["null_mean_z"]
    tol = max(0.05, 3 * float(nm.std(ddof=1)))
    assert abs(r["ref_mean_z"] - nm.mean()) <= tol, (what, f"clipped mean z: reference {r['ref_mean_z']:.3f}, "
                                                           f"nulls {np.round(nm, 3)}")
