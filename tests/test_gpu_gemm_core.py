"""The GEMM core on its own (ptts_test_gemm), against an fp64 product, on every tile layout the
product ships and on shapes the model never runs (ragged M and N, short and long K, split-K slabs,
the split tail). The interleaved-DMA tiles rely on a compiler workaround (an empty asm that pins
the next chunk's DMA addresses so no address arithmetic reuses a queued MFMA's operand registers,
DESIGN.md §4): a toolchain change that miscompiles a tile shows up here at shapes the model-level
tests never reach. The bf16-operand twins (layout + 100, engine back_mfma = BACK_BF16) are checked
against the fp64 product of the bf16-rounded operands, which they must equal up to f32 accumulation
order. The bf16x6 tiles (layout + 200, BACK_F32X6: f32 operands as exact three-piece bf16 splits,
six piece products) are checked against the fp64 product of the UNROUNDED operands, like the f32
tiles, and their error must not exceed the f32 MFMA tile's on the same operands.
Gates: f32 and bf16x6 tiles 2e-6 x sqrt(K) x max|x| x max|w| max abs; bf16 tiles the same against
the rounded operands' product."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

F32_LAYOUTS = [0, 9, 18, 20, 6, 7, 14, 23, 32, 34, 35]  # kernels.hip gemm_launch, product build
BF16_LAYOUTS = [132, 135, 131]
X6_LAYOUTS = [232, 235, 236, 239]
SHAPES = [(97, 160, 320), (200, 96, 64), (64, 64, 32), (333, 257, 544), (40, 700, 1056)]


@pytest.fixture(scope="module")
def eng():
    import pocket_tts_amd as pt

    e = pt.Engine(device=0, max_slots=1, max_ctx=64, seed=0x5EED)
    yield e
    e.close()


def bf16_round(a):
    u = np.asarray(a, np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


def operands(m, n, k, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((m, k)).astype(np.float32), rng.standard_normal((n, k)).astype(np.float32)


def check(y, ref, k):
    tol = 2e-6 * np.sqrt(k) * 4.0 * 4.0 * 4.0  # |x|, |w| <~ 4 (normal samples), margin 4
    err = float(np.abs(y.astype(np.float64) - ref).max())
    assert err <= tol, (err, tol)
    return err


@pytest.mark.parametrize("layout", F32_LAYOUTS + BF16_LAYOUTS + X6_LAYOUTS)
def test_gemm_layout_matches_fp64(eng, layout):
    worst = 0.0
    for i, (m, n, k) in enumerate(SHAPES):
        x, w = operands(m, n, k, 100 * layout + i)
        if 100 <= layout < 200:
            ref = bf16_round(x).astype(np.float64) @ bf16_round(w).astype(np.float64).T
        else:
            ref = x.astype(np.float64) @ w.astype(np.float64).T
        worst = max(worst, check(eng.test_gemm(layout, x, w), ref, k))
    print(f"layout {layout}: worst |d| {worst:.3g}")


@pytest.mark.parametrize("layout", [32, 6, 7, 132, 232])
def test_split_k_slabs_sum_to_product(eng, layout):
    m, n, k = 150, 192, 640
    x, w = operands(m, n, k, 7 + layout)
    slabs = eng.test_gemm(layout, x, w, splits=3)
    assert slabs.shape == (3, m, n)
    rx, rw = (bf16_round(x), bf16_round(w)) if 100 <= layout < 200 else (x, w)
    check(slabs.astype(np.float64).sum(0), rx.astype(np.float64) @ rw.astype(np.float64).T, k)
    # each slab is its own K slice: slab 0 covers chunks [0, 20 / 3) of the 20 32-k chunks
    c1 = 20 * 1 // 3 * 32
    check(slabs[0], rx[:, :c1].astype(np.float64) @ rw[:, :c1].astype(np.float64).T, c1)


@pytest.mark.parametrize("layout,m,n", [(34, 1024, 2092), (35, 1536, 2786)])
def test_split_tail_matches_fp64(eng, layout, m, n):
    """Tiles past whole rounds of the CUs' workgroup slots run as K slices whose last arriver sums
    them in slice order (GemmArgs::tail_S): 264 tiles of 128 x 64 on 256 slots (8 remainder tiles),
    528 on 512 (16); ragged N."""
    k = 1024
    x, w = operands(m, n, k, layout)
    y = eng.test_gemm(layout, x, w, tail_slices=4)
    check(y, x.astype(np.float64) @ w.astype(np.float64).T, k)
    # deterministic: the slice order of the sum does not depend on which slice finished last
    assert np.array_equal(y, eng.test_gemm(layout, x, w, tail_slices=4))


@pytest.mark.parametrize("m,n,k,scale", [(256, 512, 3584, 1.0), (512, 1536, 512, 1.0), (384, 640, 512, 1e-3),
                                         (200, 256, 2048, 30.0)])
def test_bf16x6_tile_is_as_accurate_as_the_f32_tile(eng, m, n, k, scale):
    """The bf16x6 tile (232) against the f32 MFMA tile (32) on the same operands, both against fp64:
    the back part's shapes (conv0 K = 3,584, Mimi qkv, a convtr) and operand scales from 1e-3 to 30.
    Gate: the split tile's RMS and max errors at most the f32 tile's (x 1.25, run-to-run margin)."""
    x, w = operands(m, n, k, k + n)
    x *= np.float32(scale)
    ref = x.astype(np.float64) @ w.astype(np.float64).T
    e32 = eng.test_gemm(32, x, w).astype(np.float64) - ref
    e6 = eng.test_gemm(232, x, w).astype(np.float64) - ref
    r32, r6 = float(np.sqrt((e32 ** 2).mean())), float(np.sqrt((e6 ** 2).mean()))
    m32, m6 = float(np.abs(e32).max()), float(np.abs(e6).max())
    print(f"K={k} scale={scale}: rms f32 {r32:.3g} bf16x6 {r6:.3g}; max f32 {m32:.3g} bf16x6 {m6:.3g}")
    assert r6 <= 1.25 * r32 and m6 <= 1.25 * m32, (r6, r32, m6, m32)
