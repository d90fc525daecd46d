"""GPU parity of each C-ABI kernel against the CPU oracle (oracle/*.py) on seeded inputs.

Integer/byte/index work must be bit-exact (preprocess, top-k, post-process
labels); fp32 arithmetic is compared with the tolerance stated per test.
"""
import hashlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    from spotter_amd._lib import lib

    assert lib().sp_device_init(0) == 0, lib().sp_last_error()
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _reset_conv_config():
    """A test that pins a tile configuration (sp_set_conv_config) leaves the by-shape choice behind."""
    yield
    from spotter_amd import ops

    ops.force_conv_config(None)


def seed(case, k=0):
    """A per-case RNG seed that does not depend on PYTHONHASHSEED (hash() of a tuple holding strings is
    randomised per process, which would make the fp32-accuracy cases draw new data every run)."""
    import zlib

    return zlib.crc32(repr(case).encode()) + k


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def conv_ref(x, w, stride, pad, scale, shift, act=None, res1=None, res2=None, row_scale=None):
    from oracle.rtdetr_np import conv2d_nhwc, gelu, relu, silu

    y = conv2d_nhwc(x.astype(np.float64).astype(np.float32), w, stride, pad).astype(np.float64)
    n, ho, wo, co = y.shape
    y = y.reshape(-1, co)
    if row_scale is not None:
        y = y * row_scale[np.arange(y.shape[0]) % row_scale.size][:, None]
    y = y * scale + shift
    if res1 is not None:
        y = y + res1
    y = y.astype(np.float32)
    if act == "relu":
        y = relu(y)
    elif act == "silu":
        y = silu(y)
    elif act == "gelu":
        y = gelu(y)
    if res2 is not None:
        y = y + res2
    return y


CONV_CASES = [
    # n, h, w, cin, cout, k, stride, act
    (2, 9, 11, 64, 96, 1, 1, "relu"),
    (1, 13, 10, 32, 40, 3, 1, "silu"),
    (2, 12, 12, 64, 64, 3, 2, None),
    (1, 17, 15, 3, 32, 3, 2, "relu"),      # stem: Cin=3 generic path
    (3, 5, 7, 128, 300, 1, 1, "gelu"),
    (1, 1, 37, 4, 512, 1, 1, "relu"),      # query_pos_head layer 0 (K=4)
    (2, 20, 20, 256, 130, 3, 1, None),     # ragged Cout
    (1, 40, 40, 96, 256, 1, 1, "relu"),    # >= 480 tiles → 128x128 path
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_matches_oracle(dev, case, workspace=None):
    from spotter_amd import ops
    from spotter_amd.ops import view

    n, h, w, cin, cout, k, st, act = case
    rng = np.random.default_rng(seed(case))
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((cout, cin, k, k)) / np.sqrt(cin * k * k)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, cout).astype(np.float32)
    sh = rng.standard_normal(cout).astype(np.float32) * 0.1
    pad = k // 2
    ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
    m = n * ho * wo
    r1 = rng.standard_normal((m, cout)).astype(np.float32)
    r2 = rng.standard_normal((m, cout)).astype(np.float32)
    ref = conv_ref(x, wt, st, pad, sc, sh, act, r1, r2)
    out = torch.empty(m * cout, device=dev)
    wk = T(wt.transpose(0, 2, 3, 1).reshape(cout, -1), dev)
    ops.conv2d(view(T(x.reshape(-1), dev), cin), n, h, w, cin, wk, cout, k, st, pad, view(out, cout),
               scale=T(sc, dev), shift=T(sh, dev), act=act, res1=view(T(r1.reshape(-1), dev), cout),
               res2=view(T(r2.reshape(-1), dev), cout), workspace=workspace)
    got = out.cpu().numpy().reshape(m, cout)
    # fp32 MFMA (exact fmaf chains) vs BLAS fp32: reassociation only
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=2e-4)


@pytest.mark.parametrize("cfg", ["220", "221", "210", "211", "120", "121", "110", "111",
                                 "4110", "4111", "4210", "4211", "4120", "4121",
                                 "1110", "1111", "1120", "1121"])
def test_conv2d_every_tile_config(dev, cfg, monkeypatch):
    """Each tile variant (sp_set_conv_config override) on a ragged 3×3 and a 1×1 with residuals."""
    from spotter_amd import ops

    ops.force_conv_config(cfg)
    for case in [(2, 11, 9, 64, 136, 3, 1, "silu"), (1, 7, 13, 96, 72, 1, 1, "relu"), (1, 9, 9, 3, 32, 3, 2, None),
                 (2, 13, 11, 32, 32, 3, 1, "relu")]:
        test_conv2d_matches_oracle(dev, case)


@pytest.mark.parametrize("case", [(1, 5, 7, 256, 96, 3, 1, "relu"), (1, 1, 300, 1024, 256, 1, 1, None),
                                  (1, 20, 20, 512, 130, 3, 1, "silu")])
def test_conv2d_split_k(dev, case):
    """Small-M / long-K launches split K over the grid when given a workspace (bs1 latency path)."""
    ws = torch.empty(4 << 20, device=dev)
    test_conv2d_matches_oracle(dev, case, workspace=ws)


SPLITK_CASES = [(1, 5, 7, 256, 96, 3, 1, "relu"), (1, 1, 300, 1024, 256, 1, 1, None), (1, 20, 20, 512, 130, 3, 1, "silu"),
                (1, 40, 40, 1024, 256, 1, 1, "relu"), (1, 40, 40, 256, 256, 3, 1, "relu")]


@pytest.mark.parametrize("mode", ["x3", "bf16"])
@pytest.mark.parametrize("cfg", ["14", "13", "16", "11", "46"])
def test_splitk_tiles_bit_identical(dev, mode, cfg):
    """Split-K launches (bs1 shapes) on the LDS-DMA tiles (sp_set_splitk_config's tile hook) give the same
    bits as the default register-staged 64×64 split-K tile: same k slices per z, same k order per element,
    the same fixed-order reduce."""
    from spotter_amd import ops
    from spotter_amd.ops import view

    ws = torch.empty(4 << 20, device=dev)
    for case in SPLITK_CASES:
        n, h, w, cin, cout, k, st, act = case
        rng = np.random.default_rng(seed(case))
        x = T(rng.standard_normal((n * h * w * cin,)).astype(np.float32), dev)
        wt = T((rng.standard_normal((cout, k * k * cin)) / np.sqrt(cin * k * k)).astype(np.float32), dev)
        pad = k // 2
        ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
        m = n * ho * wo
        r1 = view(T(rng.standard_normal(m * cout).astype(np.float32), dev), cout)
        sc = T(rng.uniform(0.5, 1.5, cout).astype(np.float32), dev)
        kw = {"x3": {"wt_planes": ops.split_bf16x3(wt)},
              "bf16": {"wt16": T(ops.bf16_bits(wt.cpu().numpy()).view(np.int16), dev)}}[mode]
        outs = []
        for c in (None, cfg):
            ops.force_splitk_config(c)
            try:
                out = torch.full((m * cout,), float("nan"), device=dev)
                ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, k, st, pad, view(out, cout), scale=sc, act=act,
                           res1=r1, workspace=ws, **kw)
                outs.append(out.cpu().numpy())
            finally:
                ops.force_splitk_config(None)
        assert not np.isnan(outs[0]).any()
        assert np.array_equal(outs[1], outs[0]), (case, mode, cfg)


@pytest.mark.parametrize("mode", ["f32", "x3", "bf16"])
def test_splitk_in_launch_combine_bit_identical(dev, mode):
    """Split-K with arrival counters (ABI v13 sp_conv_desc.splitk_counters: the tile's last-arriving
    workgroup sums the partials in z order and applies the epilogue inside the GEMM launch) gives the bits of
    the two-launch form (partials, then splitk_reduce_kernel), on the fp32-MFMA and the register-staged split /
    bf16 tiles, with BN, residuals before and after the activation and a ragged Cout. Three launches in a row
    each leave every counter at zero, and a counter array shorter than the tile grid falls back to the reduce
    launch."""
    from spotter_amd import ops
    from spotter_amd.ops import view

    ws = torch.empty(4 << 20, device=dev)
    cnt = torch.zeros(4096, dtype=torch.int32, device=dev)
    for case in SPLITK_CASES + [(1, 12, 12, 512, 202, 3, 1, "relu")]:
        n, h, w, cin, cout, k, st, act = case
        rng = np.random.default_rng(seed(case) + 1)
        x = T(rng.standard_normal((n * h * w * cin,)).astype(np.float32), dev)
        wt = T((rng.standard_normal((cout, k * k * cin)) / np.sqrt(cin * k * k)).astype(np.float32), dev)
        pad = k // 2
        ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
        m = n * ho * wo
        r1 = view(T(rng.standard_normal(m * cout).astype(np.float32), dev), cout)
        r2 = view(T(rng.standard_normal(m * cout).astype(np.float32), dev), cout)
        sc = T(rng.uniform(0.5, 1.5, cout).astype(np.float32), dev)
        sh = T(rng.standard_normal(cout).astype(np.float32), dev)
        kw = {"f32": {}, "x3": {"wt_planes": ops.split_bf16x3(wt)},
              "bf16": {"wt16": T(ops.bf16_bits(wt.cpu().numpy()).view(np.int16), dev)}}[mode]

        def run(counters):
            out = torch.full((m * cout,), float("nan"), device=dev)
            ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, k, st, pad, view(out, cout), scale=sc, shift=sh,
                       act=act, res1=r1, res2=r2, workspace=ws, counters=counters, **kw)
            return out.cpu().numpy()

        ref = run(None)
        assert not np.isnan(ref).any()
        for _ in range(3):
            assert np.array_equal(run(cnt), ref), (case, mode)
            assert int(cnt.abs().sum()) == 0, (case, mode)
        assert np.array_equal(run(cnt[:1]), ref), (case, mode)


def _bf16(a):
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    return (((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16).astype(np.uint32).view(np.float32)


# (21-26 and 31-32, the conv_pipe / conv_pp kernels, and 70-75, the conv_x3s / conv_x3p kernels, are in diagnostic
# builds only since round 5)
MFMA16_CFGS = [None, "1", "2", "3", "4", "5", "6", "11", "12", "13", "14", "15", "16", "17", "18", "19", "20", "33",
               "34", "35", "36", "37", "38", "41", "42", "43", "44", "45", "46", "47", "48", "49", "50", "51", "62", "63",
               "64", "65"]


@pytest.mark.parametrize("case", CONV_CASES[:7] + [(1, 5, 7, 256, 96, 3, 1, "relu")])
@pytest.mark.parametrize("cfg", MFMA16_CFGS)
def test_conv2d_bf16_matches_bf16_rounded_reference(dev, case, cfg, monkeypatch):
    """bf16 MFMA path == exact math on bf16-rounded activations and weights (fp32 accumulate)."""
    from spotter_amd import ops
    from spotter_amd.engine import bf16_bits
    from spotter_amd.ops import view

    if cfg:
        ops.force_conv_config(cfg)
    n, h, w, cin, cout, k, st, act = case
    rng = np.random.default_rng(seed(case, 1))
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((cout, cin, k, k)) / np.sqrt(cin * k * k)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, cout).astype(np.float32)
    sh = rng.standard_normal(cout).astype(np.float32) * 0.1
    pad = k // 2
    ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
    m = n * ho * wo
    r1 = rng.standard_normal((m, cout)).astype(np.float32)
    ref = conv_ref(_bf16(x), _bf16(wt), st, pad, sc, sh, act, r1, None)
    out = torch.empty(m * cout, device=dev)
    wk = wt.transpose(0, 2, 3, 1).reshape(cout, -1)
    w16 = torch.from_numpy(bf16_bits(wk).view(np.int16)).to(dev)
    ws = torch.empty(4 << 20, device=dev)
    ops.conv2d(view(T(x.reshape(-1), dev), cin), n, h, w, cin, T(wk, dev), cout, k, st, pad, view(out, cout),
               scale=T(sc, dev), shift=T(sh, dev), act=act, res1=view(T(r1.reshape(-1), dev), cout), wt16=w16,
               workspace=ws)
    np.testing.assert_allclose(out.cpu().numpy().reshape(m, cout), ref, rtol=1e-3, atol=1e-3)


def _conv64(x, wt, stride, pad):
    """fp64 conv (NHWC in, [M, Cout] out) — the accuracy yardstick for the fp32 GEMM paths."""
    xt = torch.from_numpy(x.astype(np.float64)).permute(0, 3, 1, 2)
    y = torch.nn.functional.conv2d(xt, torch.from_numpy(wt.astype(np.float64)), stride=stride, padding=pad)
    return y.permute(0, 2, 3, 1).reshape(-1, wt.shape[0]).numpy()


F32X3_CASES = CONV_CASES + [(2, 20, 20, 256, 256, 3, 1, None), (4, 16, 16, 1024, 256, 1, 1, None),
                            (1, 1, 300, 8, 64, 1, 1, None), (1, 1, 777, 256, 1536, 1, 1, None)]


@pytest.mark.parametrize("case", F32X3_CASES)
@pytest.mark.parametrize("cfg", MFMA16_CFGS)
def test_conv2d_f32x3_is_fp32_accurate(dev, case, cfg, monkeypatch):
    """SP_PREC_F32X3 (3-way bf16 split, 6 MFMA products) is as accurate as the fp32 MFMA path.

    Both are compared with an fp64 convolution of the same fp32 operands: the split path's max
    error must stay within 2x the fp32 MFMA path's (an exact fmaf chain) plus 1e-6 relative to
    the output scale, and under 1e-5 of the output scale outright."""
    from spotter_amd import ops
    from spotter_amd.ops import view

    n, h, w, cin, cout, k, st, _ = case
    rng = np.random.default_rng(seed(case, 2))
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((cout, cin, k, k)) / np.sqrt(cin * k * k)).astype(np.float32)
    pad = k // 2
    ref = _conv64(x, wt, st, pad)
    m = ref.shape[0]
    wk = T(wt.transpose(0, 2, 3, 1).reshape(cout, -1), dev)
    xd = view(T(x.reshape(-1), dev), cin)
    ws = torch.empty(4 << 20, device=dev)
    outs = {}
    for mode in ("fp32", "f32x3"):
        if mode == "f32x3" and cfg:
            ops.force_conv_config(cfg)
        out = torch.empty(m * cout, device=dev)
        ops.conv2d(xd, n, h, w, cin, wk, cout, k, st, pad, view(out, cout), workspace=ws,
                   wt_planes=ops.split_bf16x3(wk) if mode == "f32x3" else None)
        outs[mode] = out.cpu().numpy().reshape(m, cout).astype(np.float64)
        ops.force_conv_config(None)
    scale = np.abs(ref).max()
    e32 = np.abs(outs["fp32"] - ref).max()
    ex3 = np.abs(outs["f32x3"] - ref).max()
    assert ex3 <= 2 * e32 + 1e-6 * scale, (ex3, e32, scale)
    assert ex3 <= 1e-5 * scale, (ex3, scale)


WINO_CASES = [
    # n, h, w, cin, cout, act
    (2, 9, 11, 64, 96, "relu"),      # odd H / W: ragged last tile row and column
    (1, 20, 20, 384, 384, "silu"),   # the CCFM RepVGG shape at 20²
    (3, 8, 6, 32, 4, None),          # Cout 4 (below every N tile)
    (1, 1, 1, 32, 64, "gelu"),       # one pixel: a single, mostly padded tile
    (2, 40, 40, 256, 256, None),     # the backbone stage-3 conv2 shape at bs2
]
WINO_CFGS = [None, "63", "33", "14", "45", "44", "246", "247"]  # + 200: the direct-store epilogue forms


@pytest.mark.parametrize("case", WINO_CASES)
@pytest.mark.parametrize("cfg", WINO_CFGS)
@pytest.mark.parametrize("wm", [2, 4])
def test_winograd_is_fp32_accurate(dev, case, cfg, wm):
    """sp_winograd_f{2,4}3_* (F(m×m,3x3): fp32 transforms + the split GEMM) against an fp64 conv of the
    same fp32 operands, under 1e-5 of the output scale outright (the bar of
    test_conv2d_f32x3_is_fp32_accurate) and against the fp32 MFMA direct conv's own max error e32:
    F(2×2) within 2·e32 (+1e-6 of the scale), F(4×4) within 5·e32 — its documented error is 3-5× the
    direct conv's (tools/wino_error_study.py)."""
    from spotter_amd import ops
    from spotter_amd.ops import view

    n, h, w, cin, cout, _ = case
    rng = np.random.default_rng(seed(case, 5))
    x = rng.standard_normal((n, h, w, cin)).astype(np.float32)
    wt = (rng.standard_normal((cout, cin, 3, 3)) / np.sqrt(cin * 9)).astype(np.float32)
    ref = _conv64(x, wt, 1, 1)
    m = ref.shape[0]
    wk_host = wt.transpose(0, 2, 3, 1)
    wk = T(wk_host.reshape(cout, -1), dev)
    xd = view(T(x.reshape(-1), dev), cin)
    out32 = torch.empty(m * cout, device=dev)
    ops.conv2d(xd, n, h, w, cin, wk, cout, 3, 1, 1, view(out32, cout))
    planes = T(ops.split_bf16x3_host(ops.winograd_weights_host(wk_host, wm)), dev)
    tiles = n * ((h + wm - 1) // wm) * ((w + wm - 1) // wm)
    work = torch.full(((wm + 2) ** 2 * tiles * (cin + cout) + 64,), float("nan"), device=dev)
    out = torch.full((m * cout,), float("nan"), device=dev)
    ops.force_conv_config(cfg)
    ops.conv2d(xd, n, h, w, cin, wk, cout, 3, 1, 1, view(out, cout), wino=(planes, work, wm))
    ops.force_conv_config(None)
    got = out.cpu().numpy().reshape(m, cout).astype(np.float64)
    e32 = np.abs(out32.cpu().numpy().reshape(m, cout) - ref).max()
    ew = np.abs(got - ref).max()
    scale = np.abs(ref).max()
    assert np.isfinite(got).all()
    assert ew <= (2 if wm == 2 else 5) * e32 + 1e-6 * scale, (ew, e32, scale)
    assert ew <= 1e-5 * scale, (ew, scale)


@pytest.mark.parametrize("wm", [2, 4])
def test_winograd_epilogue_views_and_bf16(dev, wm):
    """The Winograd path's epilogue matches the direct conv's: BN scale / shift, res1 (pre-act), act,
    res2 (post-act), an input channel slice (lda > Cin) and an output slice (ldc > Cout); and the bf16
    plane form against the bf16-rounded fp64 Winograd product."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(21)
    n, h, w, cin, cout = 2, 7, 10, 64, 48
    big = rng.standard_normal((n * h * w, 96)).astype(np.float32)
    wt = (rng.standard_normal((cout, 3, 3, cin)) / 24).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, cout).astype(np.float32)
    sh = rng.standard_normal(cout).astype(np.float32)
    r1 = rng.standard_normal((n * h * w, cout)).astype(np.float32)
    r2 = rng.standard_normal((n * h * w, cout)).astype(np.float32)
    m = n * h * w
    xd = V(T(big.reshape(-1), dev), 16, 96)
    wk = T(wt.reshape(cout, -1), dev)
    kw = dict(scale=T(sc, dev), shift=T(sh, dev), act="relu", res1=V(T(r1.reshape(-1), dev), 0, cout),
              res2=V(T(r2.reshape(-1), dev), 0, cout))
    ref = torch.zeros(m * 80, device=dev)
    ops.conv2d(xd, n, h, w, cin, wk, cout, 3, 1, 1, V(ref, 8, 80), wt_planes=ops.split_bf16x3(wk), **kw)
    u = ops.winograd_weights_host(wt, wm)
    tiles = n * ((h + wm - 1) // wm) * ((w + wm - 1) // wm)
    work = torch.empty((wm + 2) ** 2 * tiles * (cin + cout), device=dev)
    got = torch.zeros(m * 80, device=dev)
    ops.conv2d(xd, n, h, w, cin, wk, cout, 3, 1, 1, V(got, 8, 80),
               wino=(T(ops.split_bf16x3_host(u), dev), work, wm), **kw)
    g, r = got.cpu().numpy().reshape(m, 80), ref.cpu().numpy().reshape(m, 80)
    np.testing.assert_allclose(g[:, 8:8 + cout], r[:, 8:8 + cout], rtol=2e-5, atol=2e-5)
    assert np.all(g[:, :8] == 0) and np.all(g[:, 8 + cout:] == 0)
    # bf16 planes: fp32 transforms, bf16-rounded V and U, fp32 accumulate
    got16 = torch.zeros(m * 80, device=dev)
    ops.conv2d(xd, n, h, w, cin, wk, cout, 3, 1, 1, V(got16, 8, 80),
               wino=(T(ops.bf16_bits(u).reshape(1, -1).view(np.int16), dev), work, wm))
    plain = torch.zeros(m * cout, device=dev)
    ops.conv2d(xd, n, h, w, cin, wk, cout, 3, 1, 1, V(plain, 0, cout))
    d16 = got16.cpu().numpy().reshape(m, 80)[:, 8:8 + cout] - plain.cpu().numpy().reshape(m, cout)
    assert np.abs(d16).max() <= 0.05 * np.abs(plain.cpu().numpy()).max(), np.abs(d16).max()


@pytest.mark.parametrize("cfg", ["12", "14", "41", "45", "46", "47", "63", "64"])
def test_direct_store_epilogue_bit_identical(dev, cfg):
    """The split mode's slab epilogue with the outputs stored straight from the accumulators (variant 4,
    sp_set_tuning SP_TUNE_GLDS_EPILOGUE) equals the slab store pass bit for bit: 1×1 convs with BN +
    residual + relu (the bottleneck expand), BN only, an output slice (ldc > Cout), ragged M and Cout, and
    the Winograd component GEMM (batched). Untouched output columns stay untouched."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(int(cfg))
    for rows, K, N, res, ldc in ((1000, 256, 192, True, 192), (777, 128, 96, True, 112), (513, 64, 256, False, 256)):
        x = T(rng.standard_normal(rows * K).astype(np.float32), dev)
        wt = T((rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32), dev)
        kw = dict(scale=T(rng.uniform(0.5, 1.5, N).astype(np.float32), dev),
                  shift=T(rng.standard_normal(N).astype(np.float32), dev), act="relu",
                  wt_planes=ops.split_bf16x3(wt))
        if res:
            kw["res1"] = V(T(rng.standard_normal(rows * N).astype(np.float32), dev), 0, N)
        outs = []
        for mode in (None, 4):
            ops.set_tuning(ops.TUNE_GLDS_EPILOGUE, mode)
            ops.force_conv_config(cfg)
            try:
                o = torch.full((rows * ldc,), 7.0, device=dev)
                ops.conv2d(V(x, 0, K), 1, 1, rows, K, wt, N, 1, 1, 0, V(o, 0, ldc), **kw)
                outs.append(o)
            finally:
                ops.force_conv_config(None)
                ops.set_tuning(ops.TUNE_GLDS_EPILOGUE, None)
        assert torch.equal(outs[0], outs[1]), (cfg, rows, K, N)
        assert bool((outs[1].view(rows, ldc)[:, N:] == 7.0).all())
    # the Winograd component GEMM (batched members, BN + residual in the output transform, not here)
    n, h, w, cin, cout = 2, 9, 11, 64, 96
    xw = T(rng.standard_normal(n * h * w * cin).astype(np.float32), dev)
    g = (rng.standard_normal((cout, 3, 3, cin)) / 24).astype(np.float32)
    pl = T(ops.split_bf16x3_host(ops.winograd_weights_host(g, 4)), dev)
    work = torch.empty(36 * n * 3 * 3 * (cin + cout) + 64, device=dev)
    outs = []
    for mode in (None, 4):
        ops.set_tuning(ops.TUNE_GLDS_EPILOGUE, mode)
        try:
            o = torch.full((n * h * w * cout,), float("nan"), device=dev)
            ops.conv2d(V(xw, 0, cin), n, h, w, cin, T(g.reshape(cout, -1), dev), cout, 3, 1, 1, V(o, 0, cout),
                       wino=(pl, work, 4))
            outs.append(o)
        finally:
            ops.set_tuning(ops.TUNE_GLDS_EPILOGUE, None)
    assert torch.equal(outs[0], outs[1])


def test_conv2d_bf16_a_rows_bit_identical(dev):
    """sp_conv2d with A given as bf16 rows (sp_conv_desc.A_bf16, the bf16 variant's maps) equals the launch on
    the same values as fp32 A (rounded to bf16 per fragment inside the GEMM, exactly): 1×1 and 3×3 stride-2
    convs, ragged M / Cout, residual epilogue, every LDS-DMA tile that builds the bf16-A form."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(23)
    for (n, h, w, cin, cout, k, stride) in [(2, 9, 13, 64, 96, 1, 1), (1, 17, 15, 32, 72, 3, 2),
                                             (3, 8, 8, 128, 256, 3, 1)]:
        x16, xf = _bf16_rows(rng.standard_normal((n * h * w, cin)).astype(np.float32))
        wt = (rng.standard_normal((cout, k * k * cin)) / np.sqrt(k * k * cin)).astype(np.float32)
        ho, wo = (h + 2 * (k // 2) - k) // stride + 1, (w + 2 * (k // 2) - k) // stride + 1
        res = rng.standard_normal((n * ho * wo, cout)).astype(np.float32)
        wk = T(wt, dev)
        w16 = T(ops.bf16_bits(wt).view(np.int16), dev)
        for cfg in (None, "14", "46", "45", "12", "33", "47", "63", "16", "51", "41", "44", "64", "13"):
            outs = []
            for xin in (T(xf.reshape(-1), dev), T(x16.reshape(-1), dev)):  # fp32 values, then the bf16 rows
                out = torch.full((n * ho * wo * cout,), float("nan"), device=dev)
                ops.force_conv_config(cfg)
                try:
                    ops.conv2d(V(xin, 0, cin), n, h, w, cin, wk, cout, k, stride, k // 2, V(out, 0, cout),
                               res1=V(T(res.reshape(-1), dev), 0, cout), act="relu", wt16=w16)
                except RuntimeError as e:
                    outs.append(str(e))
                    continue
                finally:
                    ops.force_conv_config(None)
                outs.append(out.cpu().numpy())
            if any(isinstance(o, str) for o in outs):
                assert cfg is not None, outs  # only a forced tile may lack the form
                continue
            assert np.array_equal(outs[0], outs[1]), (cfg, k, np.abs(outs[0] - outs[1]).max())


def _bf16_rows(a):
    """fp32 array → (int16 bf16 bit patterns, their exact fp32 values)."""
    from spotter_amd import ops

    bits = ops.bf16_bits(a)
    return bits.view(np.int16), ops._bf16_float(bits)


@pytest.mark.parametrize("k,stride,cfg", [(1, 1, None), (3, 2, None), (3, 1, "14"), (1, 1, "45"), (1, 1, "12"),
                                          (3, 1, "51"), (3, 2, "41"), (3, 1, "64"), (1, 1, "33"), (3, 1, "16")])
def test_conv2d_bf16_rows_in_and_out(dev, k, stride, cfg):
    """bf16 activation rows (ABI v10, the bf16 variant's maps): A_bf16 in, res1_bf16, res2_bf16, C_bf16 out (into a
    channel slice of a wider buffer) equal the fp32-row launch on the same bf16-representable values with
    its fp32 output rounded to bf16 (RNE) — bit for bit."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(31 + k + stride)
    n, h, w, cin, cout = 2, 11, 14, 64, 96
    ho, wo = (h + 2 * (k // 2) - k) // stride + 1, (w + 2 * (k // 2) - k) // stride + 1
    m = n * ho * wo
    x16, x32 = _bf16_rows(rng.standard_normal((n * h * w, cin)).astype(np.float32))
    r16, r32 = _bf16_rows(rng.standard_normal((m, cout)).astype(np.float32))
    q16, q32 = _bf16_rows(rng.standard_normal((m, cout)).astype(np.float32))
    wt = (rng.standard_normal((cout, k * k * cin)) / np.sqrt(k * k * cin)).astype(np.float32)
    wk = T(wt, dev)
    w16 = T(ops.bf16_bits(wt).view(np.int16), dev)
    sc, sh = T(rng.uniform(0.5, 1.5, cout).astype(np.float32), dev), T(rng.standard_normal(cout).astype(np.float32), dev)
    ops.force_conv_config(cfg)
    try:
        ref = torch.empty(m * cout, device=dev)
        ops.conv2d(V(T(x32.reshape(-1), dev), 0, cin), n, h, w, cin, wk, cout, k, stride, k // 2, V(ref, 0, cout),
                   scale=sc, shift=sh, act="relu", res1=V(T(r32.reshape(-1), dev), 0, cout),
                   res2=V(T(q32.reshape(-1), dev), 0, cout), wt16=w16)
        out = torch.full((m * (cout + 16),), -1, dtype=torch.int16, device=dev)
        ops.conv2d(V(T(x16.reshape(-1), dev), 0, cin), n, h, w, cin, wk, cout, k, stride, k // 2,
                   V(out, 8, cout + 16), scale=sc, shift=sh, act="relu", res1=V(T(r16.reshape(-1), dev), 0, cout),
                   res2=V(T(q16.reshape(-1), dev), 0, cout), wt16=w16)
    finally:
        ops.force_conv_config(None)
    want = ops.bf16_bits(ref.cpu().numpy()).view(np.int16).reshape(m, cout)
    got = out.cpu().numpy().reshape(m, cout + 16)
    assert np.array_equal(got[:, 8:8 + cout], want)
    assert np.all(got[:, :8] == -1) and np.all(got[:, 8 + cout:] == -1)


@pytest.mark.parametrize("cout,act,hw", [(32, "relu", (13, 70)), (64, "relu", (9, 129)), (64, None, (4, 64)),
                                         (32, None, (1, 1))])
def test_conv3x3_c32_bf16_direct(dev, cout, act, hw):
    """sp_conv3x3_c32_bf16 (the bf16 variant's direct stem 3×3, ABI v10) equals the implicit-GEMM bf16 path on
    the same bf16 rows bit for bit: both sum the 288-deep k in (tap, 16-channel) order with the same
    v_mfma_f32_32x32x16_bf16 blocks. Ragged tile edges in both directions, one-pixel maps."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(51 + cout)
    n, (h, w) = 2, hw
    m = n * h * w
    x16, _ = _bf16_rows(rng.standard_normal((m, 32)).astype(np.float32))
    wt = (rng.standard_normal((cout, 288)) / 17).astype(np.float32)
    w16 = T(ops.bf16_bits(wt).view(np.int16), dev)
    sc, sh = T(rng.uniform(0.5, 1.5, cout).astype(np.float32), dev), T(rng.standard_normal(cout).astype(np.float32), dev)
    xd = T(x16.reshape(-1), dev)
    ref = torch.full((m * cout,), -1, dtype=torch.int16, device=dev)
    ops.force_conv_config("14")
    ops.conv2d(V(xd, 0, 32), n, h, w, 32, T(wt, dev), cout, 3, 1, 1, V(ref, 0, cout), scale=sc, shift=sh, act=act,
               wt16=w16)
    ops.force_conv_config(None)
    out = torch.full((m * cout,), -1, dtype=torch.int16, device=dev)
    ops.conv3x3_c32_bf16(V(xd, 0, 32), w16, sc, sh, V(out, 0, cout), n, h, w, cout, act=act)
    assert np.array_equal(out.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("cout,act,hw", [(32, "relu", (13, 70)), (64, "relu", (9, 129)), (64, None, (4, 64)),
                                         (32, None, (1, 1)), (64, "relu", (17, 200))])
def test_conv3x3_c32_f32_direct(dev, cout, act, hw):
    """sp_conv3x3_c32 (the fp32 modes' direct stem 3×3, ABI v10) against the fp32-MFMA implicit GEMM and an
    fp64 conv: exact fp32 products, fp32 accumulation in another order, so within a few fp32 roundings of the
    288-term sums (3e-6 of the output scale; the GEMM's own error sets the bar). Ragged tile edges in both
    directions, one-pixel maps, more tiles than CUs' worth of rows (the persistent loop's prefetch)."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(61 + cout)
    n, (h, w) = 2, hw
    m = n * h * w
    x = rng.standard_normal((n, h, w, 32)).astype(np.float32)
    wt = (rng.standard_normal((cout, 3, 3, 32)) / 17).astype(np.float32)
    sc, sh = rng.uniform(0.5, 1.5, cout).astype(np.float32), rng.standard_normal(cout).astype(np.float32)
    xd, wd, scd, shd = T(x.reshape(-1), dev), T(wt.reshape(cout, 288), dev), T(sc, dev), T(sh, dev)
    ref = torch.empty(m * cout, device=dev)
    ops.conv2d(V(xd, 0, 32), n, h, w, 32, wd, cout, 3, 1, 1, V(ref, 0, cout), scale=scd, shift=shd, act=act)
    out = torch.full((m * cout,), float("nan"), device=dev)
    ops.conv3x3_c32(V(xd, 0, 32), wd, scd, shd, V(out, 0, cout), n, h, w, cout, act=act)
    got = out.cpu().numpy().reshape(n, h, w, cout)
    xp = np.pad(x.astype(np.float64), ((0, 0), (1, 1), (1, 1), (0, 0)))
    acc = np.zeros((n, h, w, cout))
    for kh in range(3):
        for kw in range(3):
            acc += xp[:, kh:kh + h, kw:kw + w, :] @ wt[:, kh, kw, :].astype(np.float64).T
    want = acc * sc + sh
    if act:
        want = np.maximum(want, 0)
    tol = 3e-6 * np.abs(want).max()
    assert np.isfinite(got).all()
    assert np.abs(got - want).max() <= tol
    assert np.abs(got - ref.cpu().numpy().reshape(n, h, w, cout)).max() <= tol


@pytest.mark.parametrize("act,hw,lds,res", [("relu", (13, 70), (64, 64), False), (None, (9, 129), (128, 192), False),
                                            ("relu", (1, 1), (64, 128), False), ("relu", (40, 64), (64, 64), False),
                                            ("relu", (13, 70), (64, 128), True), (None, (9, 129), (128, 64), True)])
def test_conv3x3_c64_bf16_direct(dev, act, hw, lds, res):
    """sp_conv3x3_c64_bf16 (the bf16 variant's stage-0 3×3) equals the implicit-GEMM bf16 path on the same
    bf16 rows bit for bit (both sum the 576-deep k in (tap, 16-channel) order with v_mfma_f32_32x32x16_bf16
    blocks); channel-slice input / output rows, ragged tiles, one-pixel maps; columns around the slice kept."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(81)
    n, (h, w) = 2, hw
    ldx, ldy = lds
    m = n * h * w
    x16, _ = _bf16_rows(rng.standard_normal((m, 64)).astype(np.float32))
    xrows = np.zeros((m, ldx), np.int16)
    xrows[:, ldx - 64:] = x16.reshape(m, 64)
    wt = (rng.standard_normal((64, 576)) / 24).astype(np.float32)
    w16 = T(ops.bf16_bits(wt).view(np.int16), dev)
    sc, sh = T(rng.uniform(0.5, 1.5, 64).astype(np.float32), dev), T(rng.standard_normal(64).astype(np.float32), dev)
    xv = V(T(xrows.reshape(-1), dev), ldx - 64, ldx)
    ref = torch.full((m * 64,), -1, dtype=torch.int16, device=dev)
    rv = None
    if res:  # the basic block's pre-activation shortcut, bf16 rows in a wider buffer
        r16, _ = _bf16_rows(rng.standard_normal((m, 64)).astype(np.float32))
        rrows = np.zeros((m, 128), np.int16)
        rrows[:, 32:96] = r16.reshape(m, 64)
        rv = V(T(rrows.reshape(-1), dev), 32, 128)
    ops.force_conv_config("14")
    try:
        ops.conv2d(xv, n, h, w, 64, T(wt, dev), 64, 3, 1, 1, V(ref, 0, 64), scale=sc, shift=sh, act=act, wt16=w16,
                   res1=rv)
    finally:
        ops.force_conv_config(None)
    out = torch.full((m * ldy,), -1, dtype=torch.int16, device=dev)
    ops.conv3x3_c64_bf16(xv, w16, sc, sh, V(out, ldy - 64, ldy), n, h, w, act=act, res1=rv)
    rows = out.cpu().numpy().reshape(m, ldy)
    assert np.all(rows[:, :ldy - 64] == -1)
    assert np.array_equal(rows[:, ldy - 64:], ref.cpu().numpy().reshape(m, 64))



@pytest.mark.parametrize("kind", ["c32_bf16_32", "c32_bf16_64", "c32_f32_32", "c32_f32_64", "c64_bf16", "c64_bf16_res"])
def test_direct_3x3_persistent_loop_many_tiles(dev, kind):
    """The persistent direct 3×3 kernels walk several tiles per workgroup (grid capped near the CU count) and
    prefetch the next tile's halo during the MFMAs: at n = 8 of 160×160 (480 tiles of 8 rows × 64 pixels per
    Cout group, well over the grid) every tile after the first comes through that loop. Checked against the
    implicit GEMM on the same operands: bit for bit on bf16 rows, within 3e-6 of the output scale in fp32."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(91)
    n, h, w = 8, 160, 160
    m = n * h * w
    cin = 64 if kind.startswith("c64") else 32
    cout = 64 if kind.endswith(("64", "bf16", "res")) else 32
    wt = (rng.standard_normal((cout, 9 * cin)) / np.sqrt(9 * cin)).astype(np.float32)
    sc = T(rng.uniform(0.5, 1.5, cout).astype(np.float32), dev)
    sh = T(rng.standard_normal(cout).astype(np.float32), dev)
    if "f32" in kind:
        xd = T(rng.standard_normal(m * cin).astype(np.float32), dev)
        wd = T(wt, dev)
        ref = torch.empty(m * cout, device=dev)
        ops.conv2d(V(xd, 0, cin), n, h, w, cin, wd, cout, 3, 1, 1, V(ref, 0, cout), scale=sc, shift=sh, act="relu")
        out = torch.full((m * cout,), float("nan"), device=dev)
        ops.conv3x3_c32(V(xd, 0, cin), wd, sc, sh, V(out, 0, cout), n, h, w, cout, act="relu")
        r, o = ref.cpu().numpy(), out.cpu().numpy()
        assert np.isfinite(o).all() and np.abs(o - r).max() <= 3e-6 * np.abs(r).max()
        return
    x16, _ = _bf16_rows(rng.standard_normal((m, cin)).astype(np.float32))
    xd = T(x16.reshape(-1), dev)
    w16 = T(ops.bf16_bits(wt).view(np.int16), dev)
    rv = None
    if kind.endswith("res"):
        r16, _ = _bf16_rows(rng.standard_normal((m, cout)).astype(np.float32))
        rv = V(T(r16.reshape(-1), dev), 0, cout)
    ref = torch.full((m * cout,), -1, dtype=torch.int16, device=dev)
    ops.force_conv_config("14")
    try:
        ops.conv2d(V(xd, 0, cin), n, h, w, cin, T(wt, dev), cout, 3, 1, 1, V(ref, 0, cout), scale=sc, shift=sh,
                   act="relu", wt16=w16, res1=rv)
    finally:
        ops.force_conv_config(None)
    out = torch.full((m * cout,), -1, dtype=torch.int16, device=dev)
    if cin == 32:
        ops.conv3x3_c32_bf16(V(xd, 0, cin), w16, sc, sh, V(out, 0, cout), n, h, w, cout, act="relu")
    else:
        ops.conv3x3_c64_bf16(V(xd, 0, cin), w16, sc, sh, V(out, 0, cout), n, h, w, act="relu", res1=rv)
    assert np.array_equal(out.cpu().numpy(), ref.cpu().numpy())

def test_pools_and_stem_bf16_rows(dev):
    """sp_maxpool3x3s2_bf16 / sp_avgpool2x2_ceil_bf16 / sp_stem_conv3x3s2_nchw_bf16 (ABI v10) equal the fp32
    kernels on the same bf16-representable inputs with the result rounded to bf16 (max: exact)."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(41)
    n, h, w, c = 2, 13, 10, 64
    x16, x32 = _bf16_rows(rng.standard_normal((n * h * w, c)).astype(np.float32))
    for fn, (ho, wo) in ((ops.maxpool3x3s2, ((h - 1) // 2 + 1, (w - 1) // 2 + 1)),
                         (ops.avgpool2x2_ceil, ((h + 1) // 2, (w + 1) // 2))):
        ref = torch.empty(n * ho * wo * c, device=dev)
        fn(T(x32.reshape(-1), dev), ref, n, h, w, c)
        out = torch.full((n * ho * wo * (c + 8),), -1, dtype=torch.int16, device=dev)
        fn(T(x16.reshape(-1), dev), V(out, 8, c + 8), n, h, w, c)
        want = ops.bf16_bits(ref.cpu().numpy()).view(np.int16).reshape(-1, c)
        got = out.cpu().numpy().reshape(-1, c + 8)
        assert np.array_equal(got[:, 8:], want), fn.__name__
        assert np.all(got[:, :8] == -1)
    # nearest ×2 upsample of bf16 rows between channel slices (a copy: bit-exact)
    up_in = T(x16.reshape(-1), dev)
    up = torch.full((n * 4 * h * w * (c + 16),), -1, dtype=torch.int16, device=dev)
    ops.upsample2x(V(up_in, 0, c), V(up, 8, c + 16), n, h, w, c)
    u = up.cpu().numpy().reshape(n, 2 * h, 2 * w, c + 16)
    src = x16.reshape(n, h, w, c)
    assert np.array_equal(u[..., 8:8 + c], src.repeat(2, axis=1).repeat(2, axis=2))
    assert np.all(u[..., :8] == -1) and np.all(u[..., 8 + c:] == -1)
    px = T(rng.uniform(0, 1, (2, 3, 37, 30)).astype(np.float32), dev)
    wt = T((rng.standard_normal((32, 27)) / 5).astype(np.float32), dev)
    sc, sh = T(rng.uniform(0.5, 1.5, 32).astype(np.float32), dev), T(rng.standard_normal(32).astype(np.float32), dev)
    m = 2 * 19 * 15
    ref = torch.empty(m * 32, device=dev)
    ops.stem_conv_nchw(px, wt, sc, sh, V(ref, 0, 32), 32, act="relu")
    out = torch.empty(m * 32, dtype=torch.int16, device=dev)
    ops.stem_conv_nchw(px, wt, sc, sh, V(out, 0, 32), 32, act="relu")
    assert np.array_equal(out.cpu().numpy(), ops.bf16_bits(ref.cpu().numpy()).view(np.int16))


def test_conv2d_f32x3_epilogue_and_views(dev):
    """The split path shares the fused epilogue: BN, residuals, act, A2, row mask, grouped rows."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(8)
    rows, K, N = 150, 64, 96
    big = rng.standard_normal((rows, 160)).astype(np.float32)
    a2 = rng.standard_normal((rows, K)).astype(np.float32)
    wt = (rng.standard_normal((N, K)) / 8).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    mask = (rng.uniform(size=50) > 0.3).astype(np.float32)
    x = big[:, 32:32 + K] + a2
    ref = ((x @ wt.T) * mask[np.arange(rows) % 50][:, None] + b).astype(np.float32)
    out = torch.zeros(3 * 70 * N, device=dev)
    wd = T(wt, dev)
    ops.conv2d(V(T(big.reshape(-1), dev), 32, 160), 1, 1, rows, K, wd, N, 1, 1, 0,
               V(out, 11 * N, N), shift=T(b, dev), a2=V(T(a2.reshape(-1), dev), 0, K),
               row_scale=T(mask, dev), rows_per_group=50, group_stride=70 * N, wt_planes=ops.split_bf16x3(wd))
    got = out.cpu().numpy().reshape(3, 70, N)[:, 11:61].reshape(rows, N)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
    assert np.all(out.cpu().numpy().reshape(3, 70, N)[:, :11] == 0)


def test_conv2d_strided_views_rowscale_a2_grouped(dev):
    """lda > Cin input slice, A2 addend, row mask, grouped output rows (source_flatten write)."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(7)
    rows, K, N = 150, 64, 96
    big = rng.standard_normal((rows, 160)).astype(np.float32)
    a2 = rng.standard_normal((rows, K)).astype(np.float32)
    wt = (rng.standard_normal((N, K)) / 8).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    mask = (rng.uniform(size=50) > 0.3).astype(np.float32)
    x = big[:, 32:32 + K] + a2
    ref = ((x @ wt.T) * mask[np.arange(rows) % 50][:, None] + b).astype(np.float32)
    # grouped output: 3 groups of 50 rows into a [3, 70, N] buffer at row offset 11
    out = torch.zeros(3 * 70 * N, device=dev)
    ops.conv2d(V(T(big.reshape(-1), dev), 32, 160), 1, 1, rows, K, T(wt, dev), N, 1, 1, 0,
               V(out, 11 * N, N), shift=T(b, dev), a2=V(T(a2.reshape(-1), dev), 0, K),
               row_scale=T(mask, dev), rows_per_group=50, group_stride=70 * N)
    got = out.cpu().numpy().reshape(3, 70, N)[:, 11:61].reshape(rows, N)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)
    assert np.all(out.cpu().numpy().reshape(3, 70, N)[:, :11] == 0)


def test_pools_and_upsample_exact(dev):
    from oracle.rtdetr_np import avgpool2_ceil, maxpool3s2, upsample2
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(3)
    # (4100, 16, 1, 4) / (70000, 2, 1, 4): more than 65535 input rows / output row chunks, so the row-strided
    # grids loop
    # (2000, 20, 3, 8): the max pool's 4-row chunks with a partial last chunk (ho = 10)
    for (n, h, w, c) in [(2, 9, 7, 8), (1, 16, 16, 64), (3, 5, 6, 4), (4100, 16, 1, 4), (70000, 2, 1, 4),
                         (2000, 20, 3, 8)]:
        x = rng.standard_normal((n, h, w, c)).astype(np.float32)
        xt = T(x.reshape(-1), dev)
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        y = torch.empty(n * ho * wo * c, device=dev)
        ops.maxpool3x3s2(xt, y, n, h, w, c)
        np.testing.assert_array_equal(y.cpu().numpy().reshape(n, ho, wo, c), maxpool3s2(x))
        ho, wo = (h + 1) // 2, (w + 1) // 2
        y = torch.empty(n * ho * wo * c, device=dev)
        ops.avgpool2x2_ceil(xt, y, n, h, w, c)
        np.testing.assert_allclose(y.cpu().numpy().reshape(n, ho, wo, c), avgpool2_ceil(x), rtol=1e-6, atol=1e-6)
        y = torch.zeros(n * 4 * h * w * 2 * c, device=dev)
        ops.upsample2x(V(xt, 0, c), V(y, 0, 2 * c), n, h, w, c)
        got = y.cpu().numpy().reshape(n, 2 * h, 2 * w, 2 * c)
        np.testing.assert_array_equal(got[..., :c], upsample2(x))
        assert np.all(got[..., c:] == 0)


def test_nchw_to_nhwc(dev):
    from spotter_amd import ops

    x = np.random.default_rng(1).standard_normal((2, 3, 5, 7)).astype(np.float32)
    y = torch.empty(x.size, device=dev)
    ops.nchw_to_nhwc(T(x, dev), y)
    np.testing.assert_array_equal(y.cpu().numpy().reshape(2, 5, 7, 3), x.transpose(0, 2, 3, 1))


def test_pools_into_channel_slice(dev):
    """Pools writing a channel slice of a wider buffer (ldy > c): the fused bottleneck shortcut's layout."""
    from oracle.rtdetr_np import avgpool2_ceil, maxpool3s2
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(5)
    n, h, w, c, red = 2, 9, 7, 8, 12
    x = rng.standard_normal((n, h, w, c)).astype(np.float32)
    xt = T(x.reshape(-1), dev)
    for fn, ref, (ho, wo) in ((ops.maxpool3x3s2, maxpool3s2, ((h - 1) // 2 + 1, (w - 1) // 2 + 1)),
                              (ops.avgpool2x2_ceil, avgpool2_ceil, ((h + 1) // 2, (w + 1) // 2))):
        y = torch.full((n * ho * wo * (red + c),), 7.0, device=dev)
        fn(xt, V(y, red, red + c), n, h, w, c)
        got = y.cpu().numpy().reshape(n, ho, wo, red + c)
        np.testing.assert_allclose(got[..., red:], ref(x), rtol=1e-6, atol=1e-6)
        assert np.all(got[..., :red] == 7.0)


def test_pools_past_65535_output_rows(dev):
    """n·ho > 65535 output rows: the pools clamp gridDim.y and stride over rows (elementwise.hip), here
    with 66000 rows (n = 33000, h = 3), into a channel slice of a wider buffer."""
    from oracle.rtdetr_np import avgpool2_ceil, maxpool3s2
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(9)
    n, h, w, c, red = 33000, 3, 2, 4, 4
    x = rng.standard_normal((n, h, w, c)).astype(np.float32)
    xt = T(x.reshape(-1), dev)
    for fn, ref, (ho, wo) in ((ops.maxpool3x3s2, maxpool3s2, ((h - 1) // 2 + 1, (w - 1) // 2 + 1)),
                              (ops.avgpool2x2_ceil, avgpool2_ceil, ((h + 1) // 2, (w + 1) // 2))):
        assert n * ho > 65535
        y = torch.full((n * ho * wo * (red + c),), 7.0, device=dev)
        fn(xt, V(y, red, red + c), n, h, w, c)
        got = y.cpu().numpy().reshape(n, ho, wo, red + c)
        np.testing.assert_allclose(got[..., red:], ref(x), rtol=1e-6, atol=1e-6)
        assert np.all(got[..., :red] == 7.0)


@pytest.mark.parametrize("case", [(1, 17, 15, 32, "relu"), (2, 640, 640, 32, "relu"), (3, 33, 8, 64, None),
                                  (1, 1, 1, 32, "relu")])
def test_stem_conv_nchw(dev, case):
    """Direct stem conv (sp_stem_conv3x3s2_nchw) from NCHW pixel_values vs the oracle conv on the
    NHWC transpose (RN:71-114 first layer: 3x3/2 pad 1, FrozenBN affine, ReLU); odd sizes cover the
    zero-padded right/bottom edges, 640² the bench shape."""
    from spotter_amd import ops
    from spotter_amd.ops import view

    n, h, w, cout, act = case
    rng = np.random.default_rng(h * 1000 + w)
    x = rng.uniform(0, 1, (n, 3, h, w)).astype(np.float32)
    wt = (rng.standard_normal((cout, 3, 3, 3)) / np.sqrt(27)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, cout).astype(np.float32)
    sh = rng.standard_normal(cout).astype(np.float32) * 0.1
    ref = conv_ref(x.transpose(0, 2, 3, 1), wt, 2, 1, sc, sh, act)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    out = torch.empty(n * ho * wo * cout, device=dev)
    wk = T(wt.transpose(0, 2, 3, 1).reshape(cout, -1), dev)
    assert ops.stem_conv_nchw(T(x, dev), wk, T(sc, dev), T(sh, dev), view(out, cout), cout, act=act) == (ho, wo)
    got = out.cpu().numpy().reshape(-1, cout)
    # sequential fp32 fmaf chain over 27 taps vs BLAS fp32: reassociation only
    np.testing.assert_allclose(got, ref, rtol=2e-4, atol=2e-4)


def test_layernorm_256_rows_views(dev):
    """The d = 256 form (four rows per wave, 16-lane groups): ragged row counts and strided row views."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(5)
    for rows in (1, 15, 17, 1001):
        x = (rng.standard_normal((rows, 320)) * 2 - 1).astype(np.float32)
        g = rng.uniform(0.5, 1.5, 256).astype(np.float32)
        b = rng.standard_normal(256).astype(np.float32)
        y = torch.full((rows * 288,), 7.0, device=dev)
        ops.layernorm(V(T(x.reshape(-1), dev), 32, 320), T(g, dev), T(b, dev), V(y, 0, 288), rows, 256)
        xs = x[:, 32:288].astype(np.float64)
        mu = xs.mean(-1, keepdims=True)
        ref = (xs - mu) / np.sqrt(((xs - mu) ** 2).mean(-1, keepdims=True) + 1e-5) * g + b
        got = y.cpu().numpy().reshape(rows, 288)
        np.testing.assert_allclose(got[:, :256], ref, rtol=1e-5, atol=1e-5)
        assert np.all(got[:, 256:] == 7.0)


def test_layernorm_bf16_rows(dev):
    """sp_layernorm_bf16 (ABI v15, the bf16 variant's encoder head): the fp32 kernel's rows rounded RNE to bf16,
    bit for bit, on ragged row counts and strided views; and LayerNorm is row-local, so normalising gathered rows
    equals gathering normalised rows (what Engine.decode relies on for the decoder's initial queries)."""
    from spotter_amd import ops
    from spotter_amd.ops import V, bf16_bits

    rng = np.random.default_rng(55)
    g = T(rng.uniform(0.5, 1.5, 256).astype(np.float32), dev)
    b = T(rng.standard_normal(256).astype(np.float32), dev)
    for rows in (1, 15, 17, 1001):
        x = T((rng.standard_normal((rows, 320)) * 2 - 1).astype(np.float32).reshape(-1), dev)
        y32 = torch.empty(rows * 256, device=dev)
        ops.layernorm(V(x, 32, 320), g, b, V(y32, 0, 256), rows, 256)
        y16 = torch.full((rows * 264,), 7, dtype=torch.int16, device=dev)
        ops.layernorm(V(x, 32, 320), g, b, V(y16, 0, 264), rows, 256)
        got = y16.cpu().numpy().reshape(rows, 264)
        assert np.array_equal(got[:, :256].view(np.uint16), bf16_bits(y32.cpu().numpy()).reshape(rows, 256))
        assert np.all(got[:, 256:] == 7)
    rows, k = 1000, 300
    x = T(rng.standard_normal((rows, 256)).astype(np.float32).reshape(-1), dev)
    idx = T(rng.permutation(rows)[:k].astype(np.int32), dev)
    full = torch.empty(rows * 256, device=dev)
    ops.layernorm(V(x, 0, 256), g, b, V(full, 0, 256), rows, 256)
    a = torch.empty(k * 256, device=dev)
    ops.gather_rows(V(full, 0, 256), rows, idx, k, 1, 256, V(a, 0, 256))
    raw = torch.empty(k * 256, device=dev)
    ops.gather_rows(V(x, 0, 256), rows, idx, k, 1, 256, V(raw, 0, 256))
    b2 = torch.empty(k * 256, device=dev)
    ops.layernorm(V(raw, 0, 256), g, b, V(b2, 0, 256), k, 256)
    assert torch.equal(a, b2)


@pytest.mark.parametrize("d", [256, 258, 384, 1000])  # 258: scalar path, 256: four rows per wave, others: float4
def test_layernorm(dev, d):
    from spotter_amd import ops
    from spotter_amd.ops import view

    rng = np.random.default_rng(d)
    x = (rng.standard_normal((77, d)) * 3 + 1).astype(np.float32)
    g = rng.uniform(0.5, 1.5, d).astype(np.float32)
    b = rng.standard_normal(d).astype(np.float32)
    y = torch.empty(77 * d, device=dev)
    ops.layernorm(view(T(x.reshape(-1), dev), d), T(g, dev), T(b, dev), view(y, d), 77, d)
    mu = x.astype(np.float64).mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    ref = (x - mu) / np.sqrt(var + 1e-5) * g + b
    np.testing.assert_allclose(y.cpu().numpy().reshape(77, d), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,heads,dh", [(300, 8, 32), (400, 8, 48), (70, 2, 64), (1, 1, 32), (17, 3, 48),
                                        (1600, 8, 48), (129, 2, 32)])
def test_attention(dev, n, heads, dh):
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(n)
    B = 2
    D = heads * dh
    qkv = rng.standard_normal((B * n, 3 * D)).astype(np.float32)
    out = torch.empty(B * n * D, device=dev)
    t = T(qkv.reshape(-1), dev)
    sc = dh ** -0.5
    ops.attention(V(t, 0, 3 * D), V(t, D, 3 * D), V(t, 2 * D, 3 * D), V(out, 0, D), B, n, heads, dh, sc)
    q = qkv[:, :D].reshape(B, n, heads, dh).transpose(0, 2, 1, 3).astype(np.float64)
    k = qkv[:, D:2 * D].reshape(B, n, heads, dh).transpose(0, 2, 1, 3).astype(np.float64)
    v = qkv[:, 2 * D:].reshape(B, n, heads, dh).transpose(0, 2, 1, 3).astype(np.float64)
    s = q @ k.transpose(0, 1, 3, 2) * sc
    s = np.exp(s - s.max(-1, keepdims=True))
    a = s / s.sum(-1, keepdims=True)
    ref = (a @ v).transpose(0, 2, 1, 3).reshape(B * n, D)
    np.testing.assert_allclose(out.cpu().numpy().reshape(B * n, D), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("n,heads,dh", [(400, 8, 32), (300, 8, 32), (1600, 8, 48), (77, 2, 64)])
def test_attention_bf16(dev, n, heads, dh):
    """sp_attention_bf16 (the bf16 variant's attention): Q / K / V rounded to bf16 as staged, scores, softmax and
    accumulation in fp32, the probabilities rounded to bf16 for the P·V MFMA. Against an fp64 attention of the
    bf16-rounded Q / K / V the only extra error is that rounding of P (2^-9 relative per term): within 1 % of
    the output scale; against the fp32 kernel on the unrounded inputs within 3 %."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(n + dh)
    B, D = 2, heads * dh
    qkv = rng.standard_normal((B * n, 3 * D)).astype(np.float32)
    t = T(qkv.reshape(-1), dev)
    out = torch.empty(B * n * D, device=dev)
    out32 = torch.empty(B * n * D, device=dev)
    sc = dh ** -0.5
    args = (V(t, 0, 3 * D), V(t, D, 3 * D), V(t, 2 * D, 3 * D))
    ops.attention(*args, V(out, 0, D), B, n, heads, dh, sc, bf16=True)
    ops.attention(*args, V(out32, 0, D), B, n, heads, dh, sc)
    r16 = torch.from_numpy(qkv).to(torch.bfloat16).to(torch.float64).numpy()
    q = r16[:, :D].reshape(B, n, heads, dh).transpose(0, 2, 1, 3)
    k = r16[:, D:2 * D].reshape(B, n, heads, dh).transpose(0, 2, 1, 3)
    v = r16[:, 2 * D:].reshape(B, n, heads, dh).transpose(0, 2, 1, 3)
    s = q @ k.transpose(0, 1, 3, 2) * sc
    s = np.exp(s - s.max(-1, keepdims=True))
    ref = ((s / s.sum(-1, keepdims=True)) @ v).transpose(0, 2, 1, 3).reshape(B * n, D)
    got = out.cpu().numpy().reshape(B * n, D)
    scale = np.abs(ref).max()
    assert np.isfinite(got).all()
    assert np.abs(got - ref).max() <= 1e-2 * scale, np.abs(got - ref).max() / scale
    assert np.abs(got - out32.cpu().numpy().reshape(B * n, D)).max() <= 3e-2 * scale


def test_msda_bf16_value_rows(dev):
    """sp_msda with bf16 value rows (value_bf16, ABI v10: the bf16 variant) against the fp32-row kernel on the
    same bf16-representable values: the sampling arithmetic is fp32 either way, but the two instantiations
    may contract the corner sums into fmas differently, so the bar is fp32 rounding (1e-6 of the scale)."""
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(12)
    B, Q, nH, dh, nL, nP = 2, 37, 8, 32, 3, 4
    shapes, starts, S = [(16, 12), (8, 6), (4, 3)], [0, 192, 240], 252
    D = nH * dh
    v16, v32 = _bf16_rows(rng.standard_normal((B * S, 2 * D)).astype(np.float32))
    offaw = np.concatenate([rng.standard_normal((B * Q, nH * nL * nP * 2)) * 2.0,
                            rng.standard_normal((B * Q, nH * nL * nP))], 1).astype(np.float32)
    ref = np.concatenate([rng.uniform(0.05, 0.95, (B * Q, 2)), rng.uniform(0.05, 0.6, (B * Q, 2))], 1).astype(np.float32)
    outs = []
    for vals in (v32, v16):
        out = torch.empty(B * Q * D, device=dev)
        ops.msda(V(T(vals.reshape(-1), dev), 0, 2 * D), D, V(T(offaw.reshape(-1), dev), 0, offaw.shape[1]),
                 T(ref, dev), V(out, 0, D), B, S, Q, nH, dh, shapes, starts, nP, 0.5)
        outs.append(out.cpu().numpy())
    d = np.abs(outs[0] - outs[1]).max()
    assert d <= 1e-6 * np.abs(outs[0]).max(), d


@pytest.mark.parametrize("bf16", [False, True])
def test_msda_point_sharing_kernel_is_bit_identical(dev, bf16):
    """msda_h8l_kernel (the decoder's shape: 8 heads × 32, 3 levels × 4 points; each point's location math done
    once by its owner lane and shared through LDS) against msda_vec_kernel (every lane repeats it), selected with
    sp_set_tuning(SP_TUNE_MSDA_GENERIC), including points far outside the map, in the engine's value_all layout
    (6 layers side by side): bit-identical for fp32 value rows; for bf16 rows the two instantiations contract the
    corner sums into fmas differently (as test_msda_bf16_value_rows notes), so there the bar is fp32 rounding."""
    from spotter_amd import ops
    from spotter_amd._lib import lib
    from spotter_amd.ops import V

    rng = np.random.default_rng(21)
    B, Q, nH, dh, nL, nP = 3, 300, 8, 32, 3, 4
    shapes, starts, S = [(20, 20), (10, 10), (5, 5)], [0, 400, 500], 525
    D = nH * dh
    vals = rng.standard_normal((B * S, 6 * D)).astype(np.float32)
    offaw = np.concatenate([rng.standard_normal((B * Q, nH * nL * nP * 2)) * 3.0,
                            rng.standard_normal((B * Q, nH * nL * nP)) * 2.0], 1).astype(np.float32)
    ref = np.concatenate([rng.uniform(0.0, 1.0, (B * Q, 2)), rng.uniform(0.01, 0.9, (B * Q, 2))], 1).astype(np.float32)
    value = V(T((_bf16_rows(vals)[0] if bf16 else vals).reshape(-1), dev), 0, 6 * D)  # int16 rows = bf16
    outs = []
    try:
        for generic in (1, 0):  # msda_vec_kernel, then the point-sharing kernel (the default)
            assert lib().sp_set_tuning(4, generic) == 0
            out = torch.full((B * Q * D,), float("nan"), device=dev)
            ops.msda(value, 3 * D, V(T(offaw.reshape(-1), dev), 0, offaw.shape[1]), T(ref, dev), V(out, 0, D),
                     B, S, Q, nH, dh, shapes, starts, nP, 0.5)
            outs.append(out.cpu().numpy())
    finally:
        lib().sp_set_tuning(4, 0)
    for o in outs[1:]:
        assert np.isfinite(o).all()
        if bf16:
            assert np.abs(outs[0] - o).max() <= 1e-6 * np.abs(outs[0]).max()
        else:
            assert np.array_equal(outs[0], o)


@pytest.mark.parametrize("pad", [0, 1])
def test_msda_matches_oracle(dev, pad):
    """MSDA core incl. out-of-range sampling points (zero padding) vs oracle.grid_sample_bilinear.
    pad=0: the decoder's 16-byte-aligned layout (vectorised kernel); pad=1: odd row stride (scalar kernel)."""
    from oracle.rtdetr_np import grid_sample_bilinear
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(11)
    B, Q, nH, dh, nL, nP = 2, 37, 8, 32, 3, 4
    shapes = [(16, 12), (8, 6), (4, 3)]
    starts = [0, 192, 240]
    S = 252
    D = nH * dh
    value = rng.standard_normal((B, S, 2 * D + pad)).astype(np.float32)  # two "layers" side by side
    offaw = np.concatenate([rng.standard_normal((B * Q, nH * nL * nP * 2)) * 2.0,
                            rng.standard_normal((B * Q, nH * nL * nP))], 1).astype(np.float32)
    ref = np.concatenate([rng.uniform(0.05, 0.95, (B * Q, 2)), rng.uniform(0.05, 0.6, (B * Q, 2))], 1).astype(np.float32)
    out = torch.empty(B * Q * D, device=dev)
    ops.msda(V(T(value.reshape(-1), dev), 0, 2 * D + pad), D + pad, V(T(offaw.reshape(-1), dev), 0, offaw.shape[1]),
             T(ref, dev), V(out, 0, D), B, S, Q, nH, dh, shapes, starts, nP, 0.5)
    # oracle (M2:200-215 + core M2:44-115)
    off = offaw[:, :nH * nL * nP * 2].reshape(B, Q, nH, nL * nP, 2)
    aw = offaw[:, nH * nL * nP * 2:].reshape(B, Q, nH, nL * nP).astype(np.float64)
    aw = np.exp(aw - aw.max(-1, keepdims=True))
    aw = aw / aw.sum(-1, keepdims=True)
    r = ref.reshape(B, Q, 4)
    loc = r[:, :, None, None, :2] + off * np.float32(1 / nP) * r[:, :, None, None, 2:] * np.float32(0.5)
    vv = value[:, :, D + pad:].reshape(B, S, nH, dh)
    exp = np.zeros((B, nH, Q, dh))
    for l, (h, w) in enumerate(shapes):
        vl = vv[:, starts[l]:starts[l] + h * w].reshape(B, h, w, nH, dh).transpose(0, 3, 1, 2, 4).reshape(B * nH, h, w, dh)
        lc = loc[:, :, :, l * nP:(l + 1) * nP].transpose(0, 2, 1, 3, 4).reshape(B * nH, Q, nP, 2)
        sv = grid_sample_bilinear(vl, lc.astype(np.float32)).reshape(B, nH, Q, nP, dh)
        exp += (sv * aw[:, :, :, l * nP:(l + 1) * nP].transpose(0, 2, 1, 3)[..., None]).sum(3)
    exp = exp.transpose(0, 2, 1, 3).reshape(B * Q, D)
    np.testing.assert_allclose(out.cpu().numpy().reshape(B * Q, D), exp, rtol=1e-4, atol=2e-5)


@pytest.mark.parametrize("n,k,reduce_c,ties", [(8400, 300, 1, False), (1000, 300, 80, False),
                                               (24000, 300, 1, False), (5000, 300, 1, True), (300, 300, 1, True),
                                               (36864, 512, 1, True), (36864, 512, 1, False), (33600, 300, 1, False),
                                               (10, 1, 1, False), (700, 1, 1, True), (4096, 257, 4, True)])
def test_topk_exact(dev, n, k, reduce_c, ties):
    from spotter_amd import ops
    from spotter_amd.ops import V

    rng = np.random.default_rng(n + k)
    rows = 3
    if ties:
        x = rng.integers(-20, 20, (rows, n * reduce_c)).astype(np.float32)
    else:
        x = rng.standard_normal((rows, n * reduce_c)).astype(np.float32)
    idx = torch.empty(rows * k, dtype=torch.int32, device=dev)
    vals = torch.empty(rows * k, device=dev)
    ops.topk_rows(V(T(x.reshape(-1), dev), 0, n * reduce_c), rows, n, k, idx, vals, reduce_c=reduce_c)
    red = x.reshape(rows, n, reduce_c).max(-1)
    exp = np.argsort(-red, axis=-1, kind="stable")[:, :k]
    np.testing.assert_array_equal(idx.cpu().numpy().reshape(rows, k), exp)
    np.testing.assert_array_equal(vals.cpu().numpy().reshape(rows, k), np.take_along_axis(red, exp, 1))


def test_postprocess_matches_oracle(dev):
    from oracle.rtdetr_np import post_process
    from spotter_amd import ops

    rng = np.random.default_rng(5)
    B, Q, C = 3, 300, 80
    logits = (rng.standard_normal((B, Q, C)) - 3).astype(np.float32)
    boxes = rng.uniform(0.05, 0.95, (B, Q, 4)).astype(np.float32)
    ts = np.array([[717, 1200], [640, 640], [1, 3000]], np.int32)
    sc = torch.empty(B * Q, device=dev)
    lb = torch.empty(B * Q, dtype=torch.int64, device=dev)
    bx = torch.empty(B * Q * 4, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)
    work = torch.empty(B * Q, dtype=torch.int32, device=dev)
    ops.postprocess(T(logits, dev), T(boxes, dev), T(ts, dev), Q, 0.5, sc, lb, bx, cnt, work)
    ref = post_process(logits, boxes, ts.tolist(), 0.5)
    sc, lb, bx, cnt = sc.cpu().numpy().reshape(B, Q), lb.cpu().numpy().reshape(B, Q), bx.cpu().numpy().reshape(B, Q, 4), cnt.cpu().numpy()
    for i in range(B):
        n = cnt[i]
        assert n == len(ref[i]["scores"])
        np.testing.assert_array_equal(lb[i, :n], ref[i]["labels"])
        np.testing.assert_allclose(sc[i, :n], ref[i]["scores"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(bx[i, :n], ref[i]["boxes"], rtol=1e-6, atol=1e-4)


PRE_SIZES = [(480, 800), (333, 517), (640, 640), (300, 200), (1080, 1920), (717, 1200), (2160, 3840),
             (1, 1), (2, 3000), (700, 640)]


@pytest.mark.parametrize("out", [640, 1280])
def test_preprocess_bit_exact(dev, out):
    from oracle.pil_resize import preprocess
    from spotter_amd import ops
    from spotter_amd.synthetic import synthetic_image

    imgs = [synthetic_image(h * 7 + w, h, w) for (h, w) in PRE_SIZES]
    res = torch.empty(len(imgs) * 3 * out * out, device=dev)
    ops.preprocess_u8([T(im, dev) for im in imgs], res, out, out)
    got = res.cpu().numpy().reshape(len(imgs), 3, out, out)
    for i, im in enumerate(imgs):
        np.testing.assert_array_equal(got[i], preprocess(im, (out, out)), err_msg=str(PRE_SIZES[i]))


@pytest.mark.parametrize("oh,ow", [(640, 640), (300, 517), (77, 1000), (1280, 700), (5, 3)])
def test_preprocess_unaligned_sources_and_ragged_column_tiles(dev, oh, ow):
    """Sources carved out of one uint8 buffer at odd byte offsets (so no row starts 4-byte aligned and the last
    image ends at the buffer's end: the dword windows' clamp), odd widths, output widths that are not a multiple
    of the 256-column tile, a single-image launch; bit-exact with the Pillow oracle."""
    from oracle.pil_resize import preprocess
    from spotter_amd import ops
    from spotter_amd.synthetic import synthetic_image

    sizes = [(717, 1200), (33, 2999), (640, 641), (1, 7), (1080, 1920)]
    imgs = [synthetic_image(13 * h + w, h, w) for h, w in sizes]
    offs, pos = [], 3
    for im in imgs:
        offs.append(pos)
        pos += im.size + 1
    pos -= 1  # the last image ends exactly at the end of the buffer
    buf = np.zeros(pos, np.uint8)
    for o, im in zip(offs, imgs):
        buf[o:o + im.size] = im.reshape(-1)
    dbuf = T(buf, dev)
    views = [dbuf[o:o + im.size].view(im.shape) for o, im in zip(offs, imgs)]
    want = [preprocess(im, (oh, ow)) for im in imgs]
    for batch, exp in ((views, want), (views[-1:], want[-1:])):
        res = torch.empty(len(batch) * 3 * oh * ow, device=dev)
        ops.preprocess_u8(batch, res, oh, ow)
        got = res.cpu().numpy().reshape(len(batch), 3, oh, ow)
        for i, e in enumerate(exp):
            np.testing.assert_array_equal(got[i], e, err_msg=str(batch[i].shape))


@pytest.mark.parametrize("out", [640, 1280, 36])
def test_preprocess_same_size_fast_path(dev, out):
    """A batch whose sources all have the output size takes the rescale + CHW kernel (Pillow returns the
    image unchanged there); bit-exact with the oracle like the resampling path."""
    from oracle.pil_resize import preprocess
    from spotter_amd import ops
    from spotter_amd.synthetic import synthetic_image

    imgs = [synthetic_image(900 + i, out, out) for i in range(3)]
    res = torch.empty(len(imgs) * 3 * out * out, device=dev)
    ops.preprocess_u8([T(im, dev) for im in imgs], res, out, out)
    got = res.cpu().numpy().reshape(len(imgs), 3, out, out)
    for i, im in enumerate(imgs):
        np.testing.assert_array_equal(got[i], preprocess(im, (out, out)))


def test_preprocess_matches_golden_digests(dev):
    """sha256 of the HF processor's pixel_values (tests/golden/preprocess.npz) — incl. test_pic.jpg."""
    from PIL import Image

    from spotter_amd import ops
    from spotter_amd.synthetic import synthetic_image

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "preprocess.npz"))
    with Image.open(os.path.join(os.path.dirname(__file__), "golden", "test_pic.jpg")) as im:
        pic = np.asarray(im.convert("RGB"))
    for (h, w, o), seed, dig in zip(g["sizes"], g["seeds"], g["digests"]):
        img = pic if seed < 0 else synthetic_image(int(seed), int(h), int(w))
        res = torch.empty(3 * o * o, device=dev)
        ops.preprocess_u8([T(img, dev)], res, int(o), int(o))
        assert hashlib.sha256(res.cpu().numpy().tobytes()).hexdigest() == str(dig), (h, w, o)


@pytest.mark.parametrize("rows,c,ld", [(1, 80, 80), (8400 * 2, 80, 80), (333, 7, 9), (1000, 12, 16)])
def test_rowmax(dev, rows, c, ld):
    """sp_rowmax: per-anchor class max (query selection), vectorised and scalar paths; max is exact."""
    from spotter_amd import ops
    from spotter_amd.ops import view

    rng = np.random.default_rng(rows + c)
    x = rng.standard_normal((rows, ld)).astype(np.float32)
    out = torch.empty(rows, device=dev)
    ops.rowmax(view(T(x.reshape(-1), dev), ld), rows, c, out)
    np.testing.assert_array_equal(out.cpu().numpy(), x[:, :c].max(1))


@pytest.mark.skipif("_diag" not in os.environ.get("SPOTTER_HIP_LIB", ""),
                    reason="the fused LayerNorm epilogue is in diagnostic builds only (SP_DIAG_KERNELS)")
@pytest.mark.parametrize("rows,k,n", [(1, 256, 256), (37, 1024, 256), (9600, 256, 256), (130, 384, 384),
                                      (64, 2048, 384), (33, 256, 512)])
def test_linear_fused_layernorm(dev, rows, k, n):
    """sp_conv2d with ln_gamma: Linear (+ row mask, bias, residual) → LayerNorm over the row in one launch
    (the AIFI / decoder post-norm and enc_output, M2:395-429, 856-904, 1376-1381), vs fp64."""
    from spotter_amd import ops
    from spotter_amd.ops import view

    rng = np.random.default_rng(rows * 7 + n)
    x = rng.standard_normal((rows, k)).astype(np.float32)
    w = (rng.standard_normal((n, k)) / np.sqrt(k)).astype(np.float32)
    b = rng.standard_normal(n).astype(np.float32) * 0.1
    res = rng.standard_normal((rows, n)).astype(np.float32)
    rs = (rng.uniform(0, 1, 11) > 0.3).astype(np.float32)
    g = rng.uniform(0.5, 1.5, n).astype(np.float32)
    be = rng.standard_normal(n).astype(np.float32) * 0.1
    t = (x.astype(np.float64) @ w.T.astype(np.float64)) * rs[np.arange(rows) % 11, None] + b + res
    mu = t.mean(1, keepdims=True)
    ref = (t - mu) / np.sqrt(((t - mu) ** 2).mean(1, keepdims=True) + 1e-5) * g + be
    out = torch.zeros(rows * n, device=dev)
    ops.linear(view(T(x.reshape(-1), dev), k), rows, k, T(w, dev), n, view(out, n), bias=T(b, dev),
               res1=view(T(res.reshape(-1), dev), n), row_scale=T(rs, dev), ln=(T(g, dev), T(be, dev), 1e-5))
    np.testing.assert_allclose(out.cpu().numpy().reshape(rows, n), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.skipif("_bounds" not in os.environ.get("SPOTTER_HIP_LIB", ""),
                    reason="bounds-check library only (SPOTTER_HIP_LIB=spotter_amd/_bounds/libspotter_bounds.so)")
def test_bounds_build_reports_a_violation(dev):
    """Positive control of the bounds-check build: a top-k index one past its image's rows makes
    sp_gather_rows read the next image's first row — inside the buffer, so no memory fault — and the
    SP_BCHECK there must count it, with its source unit, line, index and extent; the report then resets."""
    import ctypes

    from spotter_amd import ops
    from spotter_amd._lib import SP_BUILD_BOUNDS, lib
    from spotter_amd.ops import V

    L = lib()
    assert L.sp_build_flags() & SP_BUILD_BOUNDS
    buf = ctypes.create_string_buffer(4096)
    assert L.sp_bounds_report(buf, len(buf)) == 0  # clean before
    src_rows, d, k = 10, 8, 3
    src = torch.arange(2 * src_rows * d, dtype=torch.float32, device=dev)
    idx = torch.tensor([0, 9, src_rows, 1, 2, 3], dtype=torch.int32, device=dev)  # image 0's third index: one past
    dst = torch.empty(2 * k * d, device=dev)
    ops.gather_rows(V(src, 0, d), src_rows, idx, k, 2, d, V(dst, 0, d))
    hits = L.sp_bounds_report(buf, len(buf))
    rep = buf.value.decode()
    assert hits == d, rep  # one check per gathered element of the bad row
    assert "elementwise.hip" in rep and f"index={src_rows} extent={src_rows}" in rep, rep
    assert L.sp_bounds_report(buf, len(buf)) == 0  # reset
    np.testing.assert_array_equal(dst.view(2 * k, d)[2].cpu().numpy(), src.view(-1, d)[src_rows].cpu().numpy())


@pytest.mark.parametrize("bf16", [False, True])
def test_add_rows(dev, bf16):
    """sp_add_rows (the h + pos attention input): fp32 sums bit-exact; the bf16 form equals the fp32 sum rounded
    RNE (the numpy oracle's bf16_bits, the same rounding the bf16 GEMM loader applies), on strided rows."""
    from spotter_amd import ops
    from spotter_amd.ops import V, bf16_bits

    rng = np.random.default_rng(seed(("add_rows", bf16)))
    rows, cols, lda, ldb, ldy = 300, 256, 260, 512, 264
    a = rng.standard_normal((rows, lda)).astype(np.float32)
    b = (rng.standard_normal((rows, ldb)) * 3.0).astype(np.float32)
    want = a[:, :cols] + b[:, :cols]
    out = torch.zeros(rows * ldy, device=dev, dtype=torch.int16 if bf16 else torch.float32)
    ops.add_rows(V(T(a.reshape(-1), dev), 0, lda), V(T(b.reshape(-1), dev), 0, ldb), V(out, 0, ldy), rows, cols)
    got = out.cpu().numpy().reshape(rows, ldy)
    if bf16:
        assert np.array_equal(got[:, :cols].view(np.uint16), bf16_bits(want).reshape(rows, cols))
    else:
        assert np.array_equal(got[:, :cols], want)
    assert not got[:, cols:].any()  # nothing written past the row


@pytest.mark.parametrize("rows,n", [(1, 80), (129, 80), (5000, 91), (60000, 80), (777, 96), (300, 1)])
def test_linear_rowmax_bf16_matches_gemm_then_rowmax(dev, rows, n):
    """sp_linear_rowmax_bf16 (ABI v15: the bf16 variant's score head + class max, M2:1587-1599) equals the
    bf16-mode GEMM on the same bf16 rows followed by sp_rowmax, bit for bit (same MFMA, k order and bias fma)."""
    from spotter_amd import ops
    from spotter_amd.ops import V, view

    rng = np.random.default_rng(rows * 100 + n)
    k, lda = 256, 264
    x16, _ = _bf16_rows(rng.standard_normal((rows, lda)).astype(np.float32))
    w = (rng.standard_normal((n, k)) / 16).astype(np.float32)
    b = rng.standard_normal(n).astype(np.float32)
    xt = V(T(x16.reshape(-1), dev), 0, lda)
    wt = T(w.reshape(-1), dev)
    w16 = T(ops.bf16_bits(w).view(np.int16).reshape(-1), dev)
    bt = T(b, dev)
    logits = torch.empty(rows * n, device=dev)
    ops.linear(xt, rows, k, wt, n, view(logits, n), bias=bt, wt16=w16)
    want = torch.empty(rows, device=dev)
    ops.rowmax(view(logits, n), rows, n, want)
    got = torch.full((rows,), float("nan"), device=dev)
    ops.linear_rowmax_bf16(xt, rows, k, w16, n, bt, got)
    assert torch.equal(got, want)
