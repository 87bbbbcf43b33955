"""The 'rcp lemma' the GPU kernels rely on: for bf16 x and a bf16 scale s
in the normal range, bf16(x * r) == bf16(x / s) for every r within 1 ulp of 1/s (v_rcp_f32 is
1-ulp accurate), whenever |x/s| >= 2^-11 (smaller quotients encode to 0 in every format).
Exhaustive over all finite bf16 x for a spread of scales."""
import numpy as np


def _bf16_round(f32: np.ndarray) -> np.ndarray:
    u = f32.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32) << 16
    return r.astype(np.uint32).view(np.float32)


def test_rcp_lemma_exhaustive():
    xs = (np.arange(65536, dtype=np.uint32) << 16).view(np.float32)
    xs = xs[np.isfinite(xs)]
    rng = np.random.default_rng(0)
    sb = np.concatenate([rng.integers(0x0080, 0x7F00, 400), [0x3C00, 0x3DC8, 0x3F80, 0x4000, 0x3B88, 0x3E00, 0x0100,
                                                              0x7E00, 0x3F71, 0x3FFF]]).astype(np.uint32)
    for b in sb:
        s = np.array([b << 16], dtype=np.uint32).view(np.float32)[0]
        exact = _bf16_round(np.float32(xs / s))
        r0 = np.float32(1.0) / s
        for r in (r0, np.nextafter(r0, np.float32(np.inf)), np.nextafter(r0, np.float32(0))):
            with np.errstate(over="ignore", under="ignore"):
                approx = _bf16_round((xs * np.float32(r)).astype(np.float32))
            q = np.abs(xs / s)
            keep = (q >= 2.0 ** -11) & np.isfinite(q) & (q < 3e38)
            bad = keep & (approx != exact)
            assert not bad.any(), (hex(b), xs[bad][:4])
