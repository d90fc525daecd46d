"""Host-side wrappers of the C-ABI kernels, over torch device tensors.

Every wrapper checks, on the host and before the launch, that each operand's
addressed span lies inside its tensor's storage (a faulting kernel can take
the whole GPU node down), then calls libspotter_hip on torch's current stream.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import SpConvDesc, SpImageU8, SpMsdaDesc, call

ACT = {None: 0, "none": 0, "relu": 1, "silu": 2, "gelu": 3}

_hook = None


def set_launch_hook(hook):
    """hook(kind, launch, flops, nbytes, shape) wraps every kernel launch (bench.py HIP-event timing).

    kind is the kernel class ("conv", "msda", "attention", "preprocess", "topk", "layernorm",
    "elementwise", "postprocess"); flops / nbytes are the launch's ALGORITHMIC work: useful
    FLOPs and compulsory HBM bytes (every operand read once, every result written once)."""
    global _hook
    _hook = hook


def _launch(kind: str, name: str, args, flops: int = 0, nbytes: int = 0, shape=None):
    if _hook is None:
        call(name, *args)
    else:
        _hook(kind, lambda: call(name, *args), flops, nbytes, shape)


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


@dataclass
class V:
    """A strided row view into a device tensor: rows of `ld` elements from `off`. float32 rows, or bf16 rows
    held as int16 bit patterns (the bf16 variant's backbone maps, `is_bf16`)."""
    t: torch.Tensor
    off: int = 0
    ld: int = 0

    @property
    def is_bf16(self) -> bool:
        return self.t.dtype == torch.int16

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + self.t.element_size() * self.off

    def need(self, rows: int, cols: int, what: str, bf16: bool = False):
        """Checked pointer to rows × cols; float32 rows unless bf16 (then int16 bit patterns)."""
        want = torch.int16 if bf16 else torch.float32
        if self.t.dtype != want or not self.t.is_cuda:
            raise TypeError(f"{what}: expected a {'bf16 (int16)' if bf16 else 'float32'} CUDA tensor")
        if not self.t.is_contiguous():
            raise ValueError(f"{what}: tensor must be contiguous")
        last = self.off + (rows - 1) * self.ld + cols if rows > 0 else self.off
        if self.off < 0 or cols > self.ld or last > self.t.numel():
            raise ValueError(f"{what}: span rows={rows} cols={cols} ld={self.ld} off={self.off} "
                             f"exceeds numel={self.t.numel()}")
        return self.ptr


def view(t: torch.Tensor, ld: int | None = None, off: int = 0) -> V:
    return V(t, off, ld if ld is not None else t.shape[-1])


def conv2d(x: V, n: int, h: int, w: int, cin: int, wt: torch.Tensor, cout: int, k: int, stride: int,
           pad: int, out: V, *, scale=None, shift=None, act=None, res1: V | None = None,
           res2: V | None = None, a2: V | None = None, row_scale: torch.Tensor | None = None,
           rows_per_group: int = 0, group_stride: int = 0, workspace: torch.Tensor | None = None,
           wt16: torch.Tensor | None = None, wt_planes: torch.Tensor | None = None, ln=None, wino=None,
           counters: torch.Tensor | None = None):
    """ln = (gamma, beta, eps): LayerNorm over each output row fused into the epilogue (fp32 weights).
    wino = (planes, work[, m]): run this 3×3 stride-1 conv as Winograd F(m×m, 3×3), m = 2 (default) or 4
    (sp_winograd_f23_* / _f43_*), on the transformed weight planes (int16 [3 or 1, (m+2)²·Cout·Cin],
    winograd_weights_host + split) with the fp32 scratch `work`; the bf16 / split operand mode follows the
    plane count.
    counters (int32, zeroed once by the caller, one per stream): split-K launches combine their partial sums
    inside the GEMM launch (sp_conv_desc.splitk_counters, ABI v13) instead of a second reduce launch.
    wt16 (int16 bit patterns of bf16 weights, same [Cout][K] layout) selects the bf16 MFMA path;
    wt_planes (int16 [3, Cout*K]: the hi / mid / lo bf16 split of the fp32 weights, split_bf16x3)
    selects the fp32-accurate 3-way-split path (SP_PREC_F32X3)."""
    ho = (h + 2 * pad - k) // stride + 1
    wo = (w + 2 * pad - k) // stride + 1
    m = n * ho * wo
    d = SpConvDesc()
    if x.is_bf16:  # bf16 activation rows: the GEMM stages them as its one bf16 A plane
        d.A_bf16 = x.need(n * h * w, cin, "conv.A", bf16=True)
    else:
        d.A = x.need(n * h * w, cin, "conv.A")
    d.lda = x.ld
    if a2 is not None:
        d.A2 = a2.need(n * h * w, cin, "conv.A2")
        d.lda2 = a2.ld
    d.N, d.H, d.W, d.Cin = n, h, w, cin
    d.KH = d.KW = k
    d.stride, d.pad, d.Ho, d.Wo = stride, pad, ho, wo
    if wt.numel() != cout * k * k * cin or not wt.is_contiguous():
        raise ValueError(f"conv weight numel {wt.numel()} != {cout}*{k}*{k}*{cin}")
    d.Wt = wt.data_ptr()
    d.Cout = cout
    for name, t in (("scale", scale), ("shift", shift)):
        if t is not None:
            if t.numel() < cout:
                raise ValueError(f"conv.{name} too short")
            setattr(d, name, t.data_ptr())
    if row_scale is not None:
        d.row_scale = row_scale.data_ptr()
        d.row_period = row_scale.numel()
    if res1 is not None:
        if res1.is_bf16:
            d.res1_bf16 = res1.need(m, cout, "conv.res1", bf16=True)
        else:
            d.res1 = res1.need(m, cout, "conv.res1")
        d.ldr1 = res1.ld
    d.act = ACT[act]
    if res2 is not None:
        if res2.is_bf16:
            d.res2_bf16 = res2.need(m, cout, "conv.res2", bf16=True)
        else:
            d.res2 = res2.need(m, cout, "conv.res2")
        d.ldr2 = res2.ld
    if rows_per_group:
        groups = (m + rows_per_group - 1) // rows_per_group
        last = out.off + (groups - 1) * group_stride + (rows_per_group - 1) * out.ld + cout
        if last > out.t.numel() or cout > out.ld:
            raise ValueError("conv.C grouped span exceeds output")
        if out.is_bf16:
            d.C_bf16 = out.ptr
        else:
            d.C = out.ptr
    elif out.is_bf16:  # bf16 output rows (RNE in the epilogue)
        d.C_bf16 = out.need(m, cout, "conv.C", bf16=True)
    else:
        d.C = out.need(m, cout, "conv.C")
    d.ldc = out.ld
    d.out_rows_per_group = rows_per_group
    d.out_group_stride = group_stride
    if wt16 is not None and wt_planes is not None:
        raise ValueError("conv: give wt16 (bf16) or wt_planes (f32x3), not both")
    if wt16 is not None:
        if wt16.numel() != cout * k * k * cin or wt16.dtype != torch.int16 or not wt16.is_contiguous():
            raise ValueError("conv bf16 weight shape/dtype mismatch")
        d.precision = 1
        d.Wt_bf16 = wt16.data_ptr()
    if wt_planes is not None:
        if (wt_planes.dim() != 2 or wt_planes.shape[0] != 3 or wt_planes.shape[1] != cout * k * k * cin
                or wt_planes.dtype != torch.int16 or not wt_planes.is_contiguous() or not wt_planes.is_cuda):
            raise ValueError("conv f32x3 weight planes must be a contiguous int16 CUDA tensor [3, Cout*K]")
        d.precision = 2
        d.Wt_bf16 = wt_planes.data_ptr()
        d.wt_plane_stride = wt_planes.shape[1]
    if ln is not None:
        g, b, eps = ln
        if wt16 is not None or wt_planes is not None:
            raise ValueError("conv: the fused LayerNorm runs on the fp32 weights")
        if g.numel() < cout or b.numel() < cout:
            raise ValueError("conv: LayerNorm gamma / beta shorter than Cout")
        d.ln_gamma, d.ln_beta, d.ln_eps = g.data_ptr(), b.data_ptr(), float(eps)
    if workspace is not None:
        assert workspace.dtype == torch.float32 and workspace.is_cuda
        d.workspace = workspace.data_ptr()
        d.workspace_elems = workspace.numel()
    if counters is not None:
        if counters.dtype != torch.int32 or not counters.is_cuda or not counters.is_contiguous():
            raise ValueError("conv: split-K counters must be a contiguous int32 CUDA tensor")
        d.splitk_counters = counters.data_ptr()
        d.splitk_counters_len = counters.numel()
    # compulsory bytes: activations at their storage width (fp32 or bf16 rows), weights in the operand form
    # the GEMM streams (fp32, one bf16 plane, or the three split planes)
    wbytes = 2 if wt16 is not None else 6 if wt_planes is not None else 4
    nbytes = (x.t.element_size() * n * h * w * cin + 4 * n * h * w * cin * (a2 is not None)
              + wbytes * cout * k * k * cin + m * cout * (out.t.element_size()
              + (res1.t.element_size() if res1 is not None else 0) + (res2.t.element_size() if res2 is not None else 0)))
    if wino is not None:
        planes, work = wino[0], wino[1]
        wm = wino[2] if len(wino) > 2 else 2
        nc = (wm + 2) ** 2
        if k != 3 or stride != 1 or pad != 1 or ln is not None or a2 is not None:
            raise ValueError("conv: Winograd needs a 3x3 stride-1 pad-1 conv without A2 / LayerNorm")
        if wm not in (2, 4):
            raise ValueError("conv: Winograd tile must be 2 or 4")
        if (planes.dim() != 2 or planes.shape[0] not in (1, 3) or planes.shape[1] != nc * cout * cin
                or planes.dtype != torch.int16 or not planes.is_contiguous() or not planes.is_cuda):
            raise ValueError(f"conv: Winograd weight planes must be int16 [1 or 3, {nc}*Cout*Cin]")
        tiles = n * ((h + wm - 1) // wm) * ((w + wm - 1) // wm)
        if work.dtype != torch.float32 or not work.is_cuda or work.numel() < wino_work_elems(wm, tiles, cin, cout):
            raise ValueError("conv: Winograd workspace too small")
        d.precision = 2 if planes.shape[0] == 3 else 1
        d.Wt_bf16 = None
        # three launches (sp_winograd_f23_input / _gemm / _output) so the launch hook times the component
        # GEMM, a batched 1x1 GEMM of 16·T rows in the conv's operand mode, apart from the transforms
        wp, wn, s = work.data_ptr(), work.numel(), stream()
        v_el, m_el = nc * tiles * cin, nc * tiles * cout
        f = f"sp_winograd_f{wm}3"
        _launch("wino_tf", f + "_input", (C.byref(d), wp, wn, s), 0, 4 * (n * h * w * cin + v_el), (m, cin, "in"))
        _launch("conv", f + "_gemm", (C.byref(d), planes.data_ptr(), planes.shape[1], wp, wn, s),
                2 * nc * tiles * cout * cin, 4 * (v_el + m_el) + 2 * planes.numel(),
                (nc * tiles, cout, cin, 1, 1, "x3" if planes.shape[0] == 3 else "bf16", "wino", m))
        _launch("wino_tf", f + "_output", (C.byref(d), wp, wn, s), 0,
                4 * (m_el + m * cout * (1 + (res1 is not None) + (res2 is not None))), (m, cout, "out"))
        return ho, wo
    _launch("conv", "sp_conv2d", (C.byref(d), stream()), 2 * m * cout * k * k * cin, nbytes,
            (m, cout, k * k * cin, k, stride, ("f32", "bf16", "x3")[d.precision] if ln is None else "f32+ln")
            + (("rows",) if x.is_bf16 else ())  # "rows": A staged from bf16 rows (tools/tune_conv.py)
            + ("epi:" + ("res" if res1 is not None else "bn" if scale is not None or shift is not None else "none"),))
    return ho, wo


def wino_work_elems(wm: int, tiles: int, cin: int, cout: int) -> int:
    """fp32 workspace of one Winograd F(wm×wm, 3×3) conv (winograd.hip): V then M."""
    nc = (wm + 2) ** 2
    return nc * tiles * (cin + cout)


def linear(x: V, rows: int, k: int, wt: torch.Tensor, n: int, out: V, *, bias=None, act=None,
           res1: V | None = None, res2: V | None = None, a2: V | None = None, row_scale=None,
           scale=None, workspace=None, wt16=None, wt_planes=None, ln=None, counters=None):
    return conv2d(x, 1, 1, rows, k, wt, n, 1, 1, 0, out, scale=scale, shift=bias, act=act, res1=res1,
                  res2=res2, a2=a2, row_scale=row_scale, workspace=workspace, wt16=wt16, wt_planes=wt_planes,
                  ln=ln, counters=counters)


def bf16_bits(a) -> np.ndarray:
    """fp32 → bf16 bit patterns (uint16), round to nearest even (finite inputs; weights are)."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def _bf16_float(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


def split_bf16x3_host(w) -> np.ndarray:
    """fp32 weights (host) → int16 [3, numel] bf16 bit planes hi, mid, lo with w == hi + mid + lo
    (RNE at each step; both residuals are exact in fp32): the operand format of SP_PREC_F32X3.
    Host numpy at weight-pack time: no device arithmetic outside the HIP kernels."""
    w = np.ascontiguousarray(w, dtype=np.float32).reshape(-1)
    hi = bf16_bits(w)
    r1 = w - _bf16_float(hi)
    mid = bf16_bits(r1)
    lo = bf16_bits(r1 - _bf16_float(mid))
    return np.stack([hi, mid, lo]).view(np.int16)


# Winograd F(m×m, 3×3) transform matrices (winograd.hip): F(2×2) on the points (0, 1, -1, ∞); F(4×4) on
# (0, -1, 1, ½, -2, ∞), chosen for fp32 error. Bᵀ and Aᵀ are what the kernels apply (dyadic, exact in fp32);
# G is applied here in fp64.
WINO_BT = {2: np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], np.float64),
           4: np.array([[1, -1.5, -2, 1.5, 1, 0], [0, 1, -2.5, 0.5, 1, 0], [0, -1, 0.5, 2.5, 1, 0],
                        [0, -2, -1, 2, 1, 0], [0, 0.5, -1, -0.5, 1, 0], [0, 1, -1.5, -2, 1.5, 1]], np.float64)}
WINO_AT = {2: np.array([[1, 1, 1, 0], [0, 1, -1, -1]], np.float64),
           4: np.array([[1, 1, 1, 1, 1, 0], [0, -1, 1, 0.5, -2, 0], [0, 1, 1, 0.25, 4, 0],
                        [0, -1, 1, 0.125, -8, 1]], np.float64)}
WINO_G = {2: np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], np.float64),
          4: np.array([[1, 0, 0], [-1 / 3, 1 / 3, -1 / 3], [1 / 3, 1 / 3, 1 / 3], [-16 / 15, -8 / 15, -4 / 15],
                       [1 / 15, -2 / 15, 4 / 15], [0, 0, 1]], np.float64)}


def winograd_weights_host(wk, m: int = 2) -> np.ndarray:
    """3×3 conv weights [Cout][3][3][Cin] (host fp32) → the F(m×m, 3×3) transformed weights U_ab = G g Gᵀ
    as fp32 [(m+2)², Cout, Cin] (component ab = (m+2)·a + b), computed in fp64 and rounded once
    (sp_winograd_f23_* / sp_winograd_f43_*)."""
    g = np.asarray(wk, dtype=np.float64)
    if g.ndim != 4 or g.shape[1:3] != (3, 3):
        raise ValueError(f"winograd weights: expected [Cout, 3, 3, Cin], got {g.shape}")
    G = WINO_G[m]
    u = np.einsum("ai,oijc,bj->aboc", G, g, G)
    return np.ascontiguousarray(u.reshape((m + 2) ** 2, g.shape[0], g.shape[3]).astype(np.float32))


def split_bf16x3(w: torch.Tensor) -> torch.Tensor:
    """split_bf16x3_host of a (device) fp32 tensor, uploaded to the tensor's device (tests / tools)."""
    return torch.from_numpy(split_bf16x3_host(w.detach().cpu().numpy())).to(w.device)


def force_conv_config(cfg=None):
    """Tests / tuning tools: pin the GEMM tile configuration of this thread's later conv2d calls
    (sp_set_conv_config); None restores the by-shape production choice."""
    from ._lib import lib

    lib().sp_set_conv_config(-1 if cfg in (None, "", "-") else int(cfg))


def force_splitk_config(cfg=None, max_splits=None, min_ktiles=None):
    """Tuning tools: pin the tile configuration of this thread's later split-K launches only, cap their
    split-K factor and set the fewest k-tiles that split (sp_set_splitk_config); None restores the default."""
    from ._lib import lib

    lib().sp_set_splitk_config(-1 if cfg in (None, "", "-") else int(cfg), 0 if max_splits is None else int(max_splits),
                               0 if min_ktiles is None else int(min_ktiles))


TUNE_GLDS_EPILOGUE = 3  # include/spotter_hip.h sp_tuning_knob


def set_tuning(knob: int, value: int | None):
    """Tuning tools: set a knob of this thread's later launches (sp_set_tuning); None = the product default."""
    from ._lib import call

    call("sp_set_tuning", int(knob), -1 if value is None else int(value))


def nchw_to_nhwc(x: torch.Tensor, y: torch.Tensor):
    n, c, h, w = x.shape
    assert y.numel() >= x.numel() and x.is_contiguous()
    _launch("elementwise", "sp_nchw_to_nhwc", (x.data_ptr(), y.data_ptr(), n, c, h, w, stream()), 0,
            8 * x.numel())


def stem_conv_nchw(x: torch.Tensor, wt: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, y: V,
                   cout: int, act=None):
    """Backbone stem conv 1 (RN:71-114: 3x3/2, Cin 3, FrozenBN, ReLU) from NCHW pixel_values x [n,3,h,w]
    into NHWC rows y [n*ho*wo, cout] (dense rows: y.ld == cout). Direct VALU kernel, no transpose pass."""
    n, c, h, w = x.shape
    if c != 3 or x.dtype != torch.float32 or not x.is_contiguous() or not x.is_cuda:
        raise ValueError("stem_conv_nchw: x must be a contiguous float32 CUDA tensor [n,3,h,w]")
    if cout not in (32, 64) or y.ld != cout:
        raise ValueError("stem_conv_nchw: cout must be 32 or 64 with dense output rows")
    if wt.numel() != cout * 27 or scale.numel() < cout or shift.numel() < cout:
        raise ValueError("stem_conv_nchw: weight / affine size mismatch")
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    m = n * ho * wo
    yp = y.need(m, cout, "stem.y", bf16=y.is_bf16)  # bf16 rows: the bf16 variant's backbone (RNE at the store)
    _launch("conv", "sp_stem_conv3x3s2_nchw" + ("_bf16" if y.is_bf16 else ""),
            (x.data_ptr(), wt.data_ptr(), scale.data_ptr(), shift.data_ptr(), yp, n, h, w, cout, ACT[act],
             stream()), 2 * m * cout * 27, 4 * (x.numel() + cout * 27) + y.t.element_size() * m * cout,
            (m, cout, 27, 3, 2, "direct"))
    return ho, wo


def conv3x3_c32_bf16(x: V, w16: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, y: V, n: int, h: int,
                     w: int, cout: int, act=None):
    """Stem convs 2 / 3 of the bf16 variant (RN:78-103: 3×3/1, Cin 32 → Cout 32 or 64, FrozenBN, ReLU) on dense
    bf16 NHWC rows: the direct LDS-halo kernel sp_conv3x3_c32_bf16."""
    if not (x.is_bf16 and y.is_bf16) or x.ld != 32 or y.ld != cout or x.off % 8 or y.off % 8:
        raise ValueError("conv3x3_c32_bf16: dense bf16 rows (ld 32 in, Cout out) expected")
    if w16.dtype != torch.int16 or w16.numel() != cout * 288 or scale.numel() < cout or shift.numel() < cout:
        raise ValueError("conv3x3_c32_bf16: weight / affine size mismatch")
    m = n * h * w
    xp = x.need(m, 32, "c32.x", bf16=True)
    yp = y.need(m, cout, "c32.y", bf16=True)
    _launch("conv", "sp_conv3x3_c32_bf16", (xp, w16.data_ptr(), scale.data_ptr(), shift.data_ptr(), yp, n, h, w,
                                            cout, ACT[act], stream()),
            2 * m * cout * 288, 2 * (m * 32 + cout * 288 + m * cout), (m, cout, 288, 3, 1, "bf16-direct"))


def conv3x3_c32(x: V, wt: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, y: V, n: int, h: int, w: int,
                cout: int, act=None):
    """Stem convs 2 / 3 in the fp32 modes (RN:78-103: 3×3/1, Cin 32 → Cout 32 or 64, FrozenBN, ReLU) on dense
    fp32 NHWC rows: the direct LDS-halo kernel sp_conv3x3_c32 (fp32 MFMA)."""
    if x.is_bf16 or y.is_bf16 or x.ld != 32 or y.ld != cout:
        raise ValueError("conv3x3_c32: dense fp32 rows (ld 32 in, Cout out) expected")
    if wt.dtype != torch.float32 or wt.numel() != cout * 288 or scale.numel() < cout or shift.numel() < cout:
        raise ValueError("conv3x3_c32: weight / affine size mismatch")
    m = n * h * w
    xp = x.need(m, 32, "c32.x")
    yp = y.need(m, cout, "c32.y")
    _launch("conv", "sp_conv3x3_c32", (xp, wt.data_ptr(), scale.data_ptr(), shift.data_ptr(), yp, n, h, w, cout,
                                       ACT[act], stream()),
            2 * m * cout * 288, 4 * (m * 32 + cout * 288 + m * cout), (m, cout, 288, 3, 1, "f32-direct"))


def conv3x3_c64_bf16(x: V, w16: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, y: V, n: int, h: int,
                     w: int, act=None, res1: V | None = None):
    """The stage-0 3×3 of the bf16 variant (Cin 64 → 64) on bf16 rows (channel-slice views allowed): the direct
    LDS-halo kernel sp_conv3x3_c64_bf16."""
    if not (x.is_bf16 and y.is_bf16) or x.ld % 8 or x.off % 8 or y.ld % 8 or y.off % 8:
        raise ValueError("conv3x3_c64_bf16: 16-byte aligned bf16 row views expected")
    if w16.dtype != torch.int16 or w16.numel() != 64 * 576 or scale.numel() < 64 or shift.numel() < 64:
        raise ValueError("conv3x3_c64_bf16: weight / affine size mismatch")
    m = n * h * w
    xp = x.need(m, 64, "c64b.x", bf16=True)
    yp = y.need(m, 64, "c64b.y", bf16=True)
    rp, ldr = None, 0
    if res1 is not None:
        if not res1.is_bf16 or res1.ld % 8 or res1.off % 8:
            raise ValueError("conv3x3_c64_bf16: the residual must be 16-byte aligned bf16 rows")
        rp, ldr = res1.need(m, 64, "c64b.res", bf16=True), res1.ld
    _launch("conv", "sp_conv3x3_c64_bf16", (xp, x.ld, w16.data_ptr(), scale.data_ptr(), shift.data_ptr(), yp, y.ld,
                                            rp, ldr, n, h, w, ACT[act], stream()),
            2 * m * 64 * 576, 2 * (m * 64 + 64 * 576 + m * 64 * (2 if rp else 1)), (m, 64, 576, 3, 1, "bf16-direct"))


def _pool_out(y, m: int, c: int, what: str):
    """y: a dense tensor or a V row view (a channel slice of a wider buffer) → (ptr, ldy)."""
    if isinstance(y, V):
        if y.ld % 4 or y.off % 4 or (y.is_bf16 and (y.ld % 8 or y.off % 8)):
            raise ValueError(f"{what}: output view must be 16-byte aligned")
        return y.need(m, c, what, bf16=y.is_bf16), y.ld
    if y.numel() < m * c:
        raise ValueError(f"{what}: output too small")
    return y.data_ptr(), c


def _pool(name, x: torch.Tensor, y, n, h, w, c, ho, wo):
    """float32 rows, or bf16 rows (int16 x and y: the *_bf16 kernels)."""
    assert x.numel() >= n * h * w * c
    bf = x.dtype == torch.int16
    yv = y if isinstance(y, V) else view(y, c)
    if yv.is_bf16 != bf:
        raise TypeError(f"{name}: input and output rows must both be float32 or both bf16")
    yp, ldy = _pool_out(y, n * ho * wo, c, name + ".y")
    _launch("elementwise", name + ("_bf16" if bf else ""), (x.data_ptr(), yp, ldy, n, h, w, c, stream()), 0,
            x.element_size() * n * c * (h * w + ho * wo))
    return ho, wo


def maxpool3x3s2(x: torch.Tensor, y, n, h, w, c):
    return _pool("sp_maxpool3x3s2", x, y, n, h, w, c, (h - 1) // 2 + 1, (w - 1) // 2 + 1)


def avgpool2x2_ceil(x: torch.Tensor, y, n, h, w, c):
    return _pool("sp_avgpool2x2_ceil", x, y, n, h, w, c, (h + 1) // 2, (w + 1) // 2)


def upsample2x(x: V, y: V, n, h, w, c):
    """Nearest ×2 upsample into a row view. bf16 rows (the bf16 variant's encoder maps) are a pure copy: the
    same kernel moves them as float pairs (c / 2 "channels", row strides / 2)."""
    bf = x.is_bf16
    if y.is_bf16 != bf:
        raise TypeError("upsample: input and output rows must both be float32 or both bf16")
    xp = x.need(n * h * w, c, "upsample.x", bf16=bf)
    yp = y.need(n * 4 * h * w, c, "upsample.y", bf16=bf)
    if bf and (c % 8 or x.ld % 2 or y.ld % 2 or x.off % 2 or y.off % 2):
        raise ValueError("upsample: bf16 rows need c % 8 == 0 and even strides / offsets")
    k = 2 if bf else 1
    _launch("elementwise", "sp_upsample2x_nearest", (xp, x.ld // k, yp, y.ld // k, n, h, w, c // k, stream()), 0,
            x.t.element_size() * n * h * w * c * 5)


def layernorm(x: V, gamma, beta, y: V, rows, d, eps=1e-5):
    """y = LayerNorm(x) over d; y may hold bf16 rows (int16 patterns; d = 256 only): rounded RNE at the store."""
    xp = x.need(rows, d, "ln.x")
    yp = y.need(rows, d, "ln.y", bf16=y.is_bf16)
    _launch("layernorm", "sp_layernorm_bf16" if y.is_bf16 else "sp_layernorm",
            (xp, x.ld, gamma.data_ptr(), beta.data_ptr(), yp, y.ld, rows, d, eps, stream()), 8 * rows * d,
            (4 + y.t.element_size()) * rows * d)


def attention(q: V, k: V, v: V, o: V, batch, n, heads, dh, scale, bf16: bool = False):
    """softmax(Q Kᵀ · scale) V; bf16: the bf16-operand kernel (sp_attention_bf16, the bf16 variant)."""
    rows = batch * n
    args = (q.need(rows, heads * dh, "attn.q"), q.ld, k.need(rows, heads * dh, "attn.k"), k.ld,
            v.need(rows, heads * dh, "attn.v"), v.ld, o.need(rows, heads * dh, "attn.o"), o.ld, batch, n, heads,
            dh, scale, stream())
    # the bf16-operand kernel is its own class, priced at the bf16 MFMA peak (bench.py CLASS_BOUND)
    _launch("attention_bf16" if bf16 else "attention", "sp_attention_bf16" if bf16 else "sp_attention", args,
            4 * batch * heads * n * n * dh, 16 * rows * heads * dh, (batch, n, heads, dh))


def msda(value: V, value_col: int, off_aw: V, ref: torch.Tensor, out: V, B, S, Q, heads, head_dim,
         shapes, starts, points, offset_scale):
    d = SpMsdaDesc()
    L = len(shapes)
    if value.is_bf16:  # the bf16 variant's value rows
        d.value_bf16 = value.need(B * S, value_col + heads * head_dim, "msda.value", bf16=True)
    else:
        d.value = value.need(B * S, value_col + heads * head_dim, "msda.value")
    d.ld_value = value.ld
    d.value_col = value_col
    d.off_aw = off_aw.need(B * Q, heads * L * points * 3, "msda.off_aw")
    d.ld_off_aw = off_aw.ld
    assert ref.numel() >= B * Q * 4
    d.ref = ref.data_ptr()
    d.out = out.need(B * Q, heads * head_dim, "msda.out")
    d.ld_out = out.ld
    d.B, d.S, d.Q, d.heads, d.head_dim, d.levels, d.points = B, S, Q, heads, head_dim, L, points
    for i, ((h, w), s0) in enumerate(zip(shapes, starts)):
        d.level_h[i], d.level_w[i], d.level_start[i] = h, w, s0
    d.offset_scale = offset_scale
    # compulsory: the value rows the samples can touch — the whole value map, or, when the map is
    # larger than the 4 bilinear corners of every sample (1280²: 34.4 MB vs 14.7 MB per image), the
    # corner rows — plus offsets + weights + reference boxes per query and the output
    value_bytes = min(S, Q * L * points * 4) * heads * head_dim
    nbytes = value.t.element_size() * B * value_bytes + 4 * B * Q * (heads * L * points * 3 + 4 + heads * head_dim)
    # per sample: 4 bilinear taps (multiply-add) + the attention weight
    flops = B * Q * heads * L * points * head_dim * 10
    _launch("msda", "sp_msda", (C.byref(d), stream()), flops, nbytes,
            (B, S, Q, heads, head_dim, L, points, value.t.element_size()))


def topk_rows(x: V, rows, n, k, idx: torch.Tensor, vals: torch.Tensor | None = None, reduce_c=1,
              apply_sigmoid=False):
    xp = x.need(rows, n * reduce_c, "topk.x")
    assert idx.dtype == torch.int32 and idx.numel() >= rows * k
    if vals is not None:
        assert vals.numel() >= rows * k
    _launch("topk", "sp_topk_rows", (xp, x.ld, rows, n, reduce_c, int(apply_sigmoid), k,
                                     vals.data_ptr() if vals is not None else None, idx.data_ptr(), stream()),
            0, 4 * rows * (n * reduce_c + 2 * k), (rows, n, reduce_c, k))


def rowmax(x: V, rows, c, out: torch.Tensor):
    """out[r] = max over the first c columns of row r (query selection's per-anchor class max)."""
    assert out.dtype == torch.float32 and out.numel() >= rows
    _launch("topk", "sp_rowmax", (x.need(rows, c, "rowmax.x"), x.ld, rows, c, out.data_ptr(), stream()),
            0, 4 * rows * (c + 1), (rows, c))


def linear_rowmax_bf16(x: V, rows: int, k: int, wt16: torch.Tensor, n: int, bias: torch.Tensor, out: torch.Tensor):
    """out[r] = max_c (x[r] · W[c] + bias[c]) over n classes: bf16 rows x, bf16 weights [n, k] (the bf16 mode's
    packed linear weights) — the score head + rowmax of query selection without the logits."""
    xp = x.need(rows, k, "linear_rowmax.x", bf16=True)
    if wt16.dtype != torch.int16 or wt16.numel() < n * k or out.numel() < rows or bias.numel() < n:
        raise ValueError("linear_rowmax_bf16: weight / bias / out size")
    _launch("conv", "sp_linear_rowmax_bf16", (xp, x.ld, wt16.data_ptr(), bias.data_ptr(), rows, n, k, out.data_ptr(),
                                              stream()), 2 * rows * n * k, rows * k * 2 + n * k * 2 + rows * 4,
            (rows, n, k, 1, 1, "bf16", "rows", "rowmax"))


def gather_rows(src: V, src_rows, idx: torch.Tensor, k, batch, d, dst: V):
    sp_ = src.need(batch * src_rows, d, "gather.src")
    dp = dst.need(batch * k, d, "gather.dst")
    _launch("elementwise", "sp_gather_rows", (sp_, src.ld, src_rows, idx.data_ptr(), k, batch, d, dp, dst.ld,
                                              stream()), 0, 4 * batch * k * (2 * d + 1))


def add_rows(a: V, b: V, out: V, rows: int, cols: int):
    """out = a + b (fp32 rows in; out fp32 rows, or bf16 rows rounded RNE when out holds int16 patterns)."""
    ap = a.need(rows, cols, "add_rows.a")
    bp = b.need(rows, cols, "add_rows.b")
    if out.is_bf16:
        yp, y16 = None, out.need(rows, cols, "add_rows.out", bf16=True)
    else:
        yp, y16 = out.need(rows, cols, "add_rows.out"), None
    _launch("elementwise", "sp_add_rows", (ap, a.ld, bp, b.ld, yp, y16, out.ld, rows, cols, stream()), 0,
            rows * cols * (8 + out.t.element_size()))


def ref_init(delta: V, anchors: torch.Tensor, idx: torch.Tensor, batch, k, ref: torch.Tensor):
    dp = delta.need(batch * k, 4, "ref_init.delta")
    assert ref.numel() >= batch * k * 4
    _launch("elementwise", "sp_ref_init", (dp, delta.ld, anchors.data_ptr(), idx.data_ptr(), batch, k,
                                           ref.data_ptr(), stream()), 0, 4 * batch * k * 13)


def box_refine(delta: V, ref: torch.Tensor, rows):
    dp = delta.need(rows, 4, "box_refine.delta")
    assert ref.numel() >= rows * 4
    _launch("elementwise", "sp_box_refine", (dp, delta.ld, ref.data_ptr(), rows, stream()), 0, 4 * rows * 12)


def preprocess_u8(images, out: torch.Tensor, out_h: int, out_w: int):
    """images: list of uint8 CUDA tensors [H, W, 3] (contiguous)."""
    n = len(images)
    arr = (SpImageU8 * n)()
    for i, im in enumerate(images):
        assert im.dtype == torch.uint8 and im.is_cuda and im.dim() == 3 and im.shape[2] == 3
        assert im.is_contiguous()
        arr[i].data = im.data_ptr()
        arr[i].height, arr[i].width = im.shape[0], im.shape[1]
        arr[i].row_stride = im.shape[1] * 3
    assert out.numel() >= n * 3 * out_h * out_w and out.dtype == torch.float32
    nbytes = sum(int(im.numel()) for im in images) + 4 * n * 3 * out_h * out_w
    _launch("preprocess", "sp_preprocess_u8", (arr, n, out_h, out_w, out.data_ptr(), stream()), 0, nbytes,
            (n, out_h, out_w))


def postprocess(logits: torch.Tensor, boxes: torch.Tensor, target_hw: torch.Tensor, k: int, threshold: float,
                scores, labels, boxes_xyxy, counts, work):
    b, q, c = logits.shape
    assert logits.is_contiguous() and boxes.is_contiguous() and boxes.shape[:2] == (b, q)
    assert target_hw.dtype == torch.int32 and target_hw.numel() >= 2 * b
    assert scores.numel() >= b * k and labels.numel() >= b * k and labels.dtype == torch.int64
    assert boxes_xyxy.numel() >= b * k * 4 and counts.numel() >= b and work.numel() >= b * k
    args = (logits.data_ptr(), boxes.data_ptr(), target_hw.data_ptr(), b, q, c, k, threshold, scores.data_ptr(),
            labels.data_ptr(), boxes_xyxy.data_ptr(), counts.data_ptr(), work.data_ptr(), stream())
    _launch("postprocess", "sp_postprocess", args, 0, 4 * b * (q * c + q * 4 + k * 7), (b, q, c, k))
