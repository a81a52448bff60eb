"""Each conv kernel family against a plain PyTorch fp32 reference (F.conv2d + the epilogue), through
the C-ABI entry mlic_conv_run.  Shapes: the layer types of MLIC++ that each family serves
(g_a/g_s point convs and GDN/IGDN, subpel 3x3 convs with PixelShuffle, the N -> 12 output conv,
the 3 -> N input convs, latent-resolution context GEMMs), plus ragged pixel counts."""
import ctypes as C
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GELU, GDN, IGDN, TANH, MASK_A, MASK_N, RES, SHUFFLE, SQUARE = 1, 2, 4, 8, 16, 32, 64, 128, 256
F32, X3, X3V2, PW, NARROW, SMALLCIN, HALO, X4, X4H, AUTO = 0, 1, 2, 3, 4, 5, 6, 7, 8, -1


def reference(x, w, b, stride, epi, res):
    y = F.conv2d((x * x) if epi & SQUARE else x, w, b, stride=stride, padding=w.shape[-1] // 2)
    if epi & GELU:
        y = F.gelu(y)
    if epi & GDN:
        y = x * torch.rsqrt(y)
    if epi & IGDN:
        y = x * torch.sqrt(y)
    if epi & TANH:
        y = 0.5 * torch.tanh(y)
    if epi & (MASK_A | MASK_N):  # checkerboard: anchor cells have (h + w) odd
        hh = torch.arange(y.shape[-2], device=y.device).view(-1, 1)
        ww = torch.arange(y.shape[-1], device=y.device).view(1, -1)
        anchor = ((hh + ww) % 2) == 1
        y = y * (anchor if epi & MASK_A else ~anchor).to(y.dtype)
    if epi & SHUFFLE:
        y = F.pixel_shuffle(y, 2)
    if epi & RES:
        y = y + res
    return y


def run(impl, B, Cin, Cout, H, W, K, stride=1, epi=0, seed=0, wmul=1.0, xmul=1.0):
    from mlic_amd import _lib
    g = torch.Generator().manual_seed(seed)
    dev = torch.device("cuda")
    x = (torch.rand(B, Cin, H, W, generator=g) - 0.5).to(dev)
    w = ((torch.rand(Cout, Cin, K, K, generator=g) - 0.5) / (Cin * K * K) ** 0.5).to(dev)
    b = (torch.rand(Cout, generator=g) - 0.5).to(dev)
    x, w = x * xmul, w * wmul
    if epi & (GDN | IGDN):  # GDN: gamma >= 0, beta > 0 (compressai reparametrisation keeps them so)
        x = x * 4
        w = w.abs() * 0.1
        b = 1.0 + b.abs()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    oshape = (B, Cout // 4, 2 * Ho, 2 * Wo) if epi & SHUFFLE else (B, Cout, Ho, Wo)
    res = (torch.rand(*oshape, generator=g) - 0.5).to(dev) if epi & RES else None
    y = torch.full(oshape, float("nan"), device=dev)
    aux = x if epi & (GDN | IGDN) else None
    st = torch.cuda.current_stream().cuda_stream
    ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    _lib.call("mlic_conv_run", C.c_void_p(st), impl, ptr(x), ptr(w), ptr(b), ptr(y), B, Cin, Cout, H, W, K, stride,
              epi, ptr(aux), ptr(res))
    ref = reference(x.double(), w.double(), b.double(), stride, epi, res.double() if res is not None else None)
    return y, ref.float()


def needs_ab(impl):
    """The A/B-only families (v1 tiles, halo tiles) are only in a `make AB=1` library."""
    from mlic_amd import _lib
    if impl in (X3, HALO) and not _lib.ab_families():
        pytest.skip("A/B-only kernel family: not in the product library (make AB=1)")


def check(y, ref, rtol=2e-5):
    assert torch.isfinite(y).all(), "unwritten or non-finite outputs"
    err = (y - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= rtol * scale + 1e-6, f"max err {err:.3e} (scale {scale:.3e})"


@pytest.mark.parametrize("cin", [48, 96, 128, 160, 192])
def test_pw_resident_sizes(cin):
    check(*run(PW, 2, cin, cin, 48, 80, 1))


@pytest.mark.parametrize("epi", [0, GELU, GDN | SQUARE, IGDN | SQUARE, GELU | RES, GDN | SQUARE | RES])
def test_pw_resident_epilogues(epi):
    check(*run(PW, 2, 192, 192, 36, 60, 1, epi=epi))
    check(*run(PW, 1, 48, 48, 37, 53, 1, epi=epi))  # small-decoder width: 3 k-steps, partial co-tile


def test_pw_resident_stride2():
    check(*run(PW, 2, 192, 192, 68, 96, 1, stride=2))
    check(*run(PW, 1, 128, 128, 37, 51, 1, stride=2, epi=GELU))  # odd sizes: ragged tiles


# the latent-resolution 1x1 convs (MLICPP_L): LRP 224 -> 128 and its head 128 -> 32 (0.5 tanh,
# checkerboard mask, residual), channel-context 32i -> 192 / 192 -> 128, context q/k/v, qkv_proj,
# proj, mlp.0 / mlp.4 (+ residual) and skip
@pytest.mark.parametrize("cin,cout,epi", [
    (224, 128, GELU), (128, 32, TANH | MASK_A | RES), (128, 32, TANH | MASK_N | RES),
    (32, 192, GELU), (64, 192, GELU), (96, 192, GELU), (128, 192, GELU), (160, 192, GELU), (192, 128, GELU),
    (32, 32, 0), (64, 64, 0), (32, 96, 0), (96, 128, GELU), (64, 128, GELU), (128, 64, RES), (96, 64, 0)])
def test_pw_resident_latent(cin, cout, epi):
    check(*run(PW, 2, cin, cout, 68, 120, 1, epi=epi))
    check(*run(PW, 1, cin, cout, 37, 53, 1, epi=epi, seed=1))  # ragged: tail tile, odd width for the mask


def test_pw_resident_ragged_and_many_tiles():
    check(*run(PW, 3, 192, 192, 37, 53, 1))   # 1961 px: tail tile per image
    check(*run(PW, 2, 192, 192, 136, 240, 1))  # > 2048 tiles: every wave loops


@pytest.mark.parametrize("epi", [0, SHUFFLE])
def test_narrow(epi):
    check(*run(NARROW, 2, 192, 12, 40, 72, 3, epi=epi))
    check(*run(NARROW, 1, 96, 12, 19, 44, 3, epi=epi))    # W % 4 == 0 (float4 patch loads)
    check(*run(NARROW, 1, 192, 12, 33, 200, 3, epi=epi))  # ragged 128-column tile


@pytest.mark.parametrize("stride", [1, 2])
def test_smallcin(stride):
    check(*run(SMALLCIN, 2, 3, 192, 64, 96, 1, stride=stride))               # 4-pixel vector path
    check(*run(SMALLCIN, 2, 3, 192, 64, 96, 1, stride=stride, epi=GELU | RES))
    check(*run(SMALLCIN, 1, 3, 192, 37, 53, 1, stride=stride, epi=GELU))      # odd width: scalar path
    # 3x3 pad 1 (MLICPP_M_SMALL_DEC's dense first conv, 3 -> N stride 2): borders, both paths
    check(*run(SMALLCIN, 2, 3, 192, 64, 96, 3, stride=stride, epi=GELU))
    check(*run(SMALLCIN, 1, 3, 96, 37, 53, 3, stride=stride))


@pytest.mark.parametrize("impl", [F32, X3, X3V2])
@pytest.mark.parametrize("shape", [
    (2, 192, 768, 24, 40, 3, 1, SHUFFLE | GELU),  # subpel conv
    (2, 192, 192, 33, 47, 1, 1, GDN | SQUARE),     # GDN on the generic tiles
    (2, 960, 320, 17, 30, 1, 1, 0),                # entropy-parameters GEMM
    (2, 288, 96, 17, 30, 5, 1, 0),                 # inter-context 5x5 reprojection
    (1, 192, 192, 34, 60, 3, 2, GELU),             # strided 3x3
    (1, 96, 64, 9, 13, 3, 1, 0),                   # K-steps 27: odd count, tiny grid
    (2, 320, 256, 40, 120, 1, 1, GELU),            # (MLIC_V2_WIDE=1: 8-wave 256x256 tile)
    (2, 608, 224, 37, 120, 1, 1, RES),             # partial Cout and pixel tiles
    (2, 192, 320, 40, 121, 3, 1, 0),               # 3x3: 256-row tile + 64-row remainder launch
    (2, 640, 320, 40, 120, 1, 1, GELU | RES),      # EP 640 -> 320: split launch with residual
    (2, 192, 384, 24, 64, 3, 1, SHUFFLE),          # split launch under PixelShuffle (rows 256..383)
    (1, 32, 48, 8, 8, 1, 1, 0),                    # a single K-step
])
def test_generic_tiles(impl, shape):
    needs_ab(impl)
    B, cin, cout, H, W, K, s, epi = shape
    check(*run(impl, B, cin, cout, H, W, K, stride=s, epi=epi))


@pytest.mark.parametrize("shape", [
    (2, 192, 768, 24, 64, SHUFFLE | GELU),   # g_s subpel conv, 2 x 3 tiles
    (1, 192, 768, 19, 45, SHUFFLE),          # ragged tiles at every edge
    (2, 96, 192, 16, 32, GELU | RES),        # Cout not a multiple of 128, residual
    (1, 160, 96, 9, 40, 0),                  # Cin 160 (5 chunks), Cout < 128
    (1, 100, 100, 8, 32, GDN | SQUARE),      # Cin not a multiple of 32 (zero-padded chunk)
])
def test_halo(shape):
    needs_ab(HALO)
    B, cin, cout, H, W, epi = shape
    check(*run(HALO, B, cin, cout, H, W, 3, epi=epi))


@pytest.mark.parametrize("shape", [
    (2, 960, 320, 17, 30, 1, GELU),   # entropy-parameters 1x1 GEMM
    (1, 608, 224, 9, 45, 1, 0),       # LRP point conv, ragged
    (2, 288, 96, 17, 30, 5, 0),       # 5x5 reprojection
    (1, 64, 40, 7, 33, 5, RES),       # 5x5, 2 chunks, Cout < 64, residual
])
def test_halo_k1_k5(shape):
    needs_ab(HALO)
    B, cin, cout, H, W, K, epi = shape
    check(*run(HALO, B, cin, cout, H, W, K, epi=epi))


@pytest.mark.parametrize("shape", [
    (2, 192, 768, 24, 64, 3, SHUFFLE | GELU),   # g_s subpel conv: 3 x 256-row Cout tiles, 2 x 3 pixel tiles
    (1, 192, 768, 19, 45, 3, SHUFFLE),          # ragged pixel tiles at every edge
    (2, 320, 256, 17, 30, 3, GELU | RES),       # 10 chunks, residual
    (1, 100, 200, 9, 33, 3, 0),                 # Cin not a multiple of 32, Cout 200 (partial 256 tile)
    (2, 128, 128, 16, 40, 3, GDN | SQUARE),     # 128-row tile (Cout < 192), GDN epilogue on the packed x^2
    (2, 960, 320, 17, 30, 1, GELU),             # 1x1 GEMM (entropy parameters), partial second tile
    (1, 288, 96, 13, 37, 5, 0),                 # 5x5 reprojection, 128-row tile
    (1, 480, 1920, 8, 16, 3, SHUFFLE | GELU),   # h_s subpel 480 -> 1920, 8 Cout tiles
    (2, 800, 64, 17, 30, 1, RES),               # 64-row tile (LocalContext fusion), residual
    (1, 128, 40, 9, 37, 1, 0),                  # Cout < 64, ragged folded pixel row
    (2, 192, 192, 24, 40, 3, GELU),             # 192-row tile (4 x 2 waves of 48 rows): SD dense g_a conv
    (1, 96, 160, 19, 45, 3, RES),               # 192-row tile, 160 rows real, ragged pixel tiles
    (2, 192, 192, 16, 32, 3, GDN | SQUARE | RES),  # 192-row tile, GDN epilogue + residual
    (2, 256, 96, 17, 30, 5, 0),                 # 96-row tile (2 x 4 waves of 48 rows): context reprojection
    (2, 160, 80, 17, 30, 3, GELU | RES),        # 96-row tile, 80 rows real
    (1, 96, 96, 9, 45, 1, 0),                   # 96-row tile, 1x1, ragged folded pixel row
    (2, 640, 224, 17, 30, 1, GELU),             # 224-row tile (2 x 4 waves of 112 rows): LRP point conv
    (1, 224, 200, 9, 33, 3, RES),               # 224-row tile, 200 rows real
])
def test_x4(shape):
    B, cin, cout, H, W, K, epi = shape
    check(*run(X4, B, cin, cout, H, W, K, epi=epi))


@pytest.mark.parametrize("shape", [
    (2, 192, 768, 24, 64, 3, SHUFFLE | GELU),   # g_s subpel conv
    (1, 192, 768, 19, 45, 3, SHUFFLE),          # ragged pixel tiles at every edge (clamped halo lines)
    (1, 100, 200, 9, 33, 3, 0),                 # Cin not a multiple of 32
    (2, 192, 192, 24, 40, 3, GELU),             # 192-row tile
    (2, 256, 96, 17, 30, 5, 0),                 # 5x5, 96-row tile
    (1, 288, 96, 13, 37, 5, 0),                 # 5x5, 128-row tile, few tiles: split-K on chunk bounds
    (1, 480, 1920, 8, 16, 3, SHUFFLE | GELU),   # h_s subpel, few tiles: split-K
])
def test_x4_halo_vs_per_tap(shape):
    """conv_x4's halo-staged B operand (one (8+K-1) x (32+K-1) image per 32-channel chunk, every tap a
    shifted read of it) against B staged per tap: the same operands in the same MFMA order, so the
    outputs are bit-identical when the K loop is not split (the default); with split-K forced on
    (few-tile shapes) the halo form splits on chunk boundaries, so both are checked against float64
    and against the unsplit result to the float64 tolerance."""
    from mlic_amd import _lib
    B, cin, cout, H, W, K, epi = shape
    res = {}
    try:
        for split in (0, 1):
            _lib.call("mlic_set_kernel_option", b"x4_splitk", split)
            for halo in (1, 0):
                _lib.call("mlic_set_kernel_option", b"x4_halo", halo)
                res[(split, halo)] = run(X4, B, cin, cout, H, W, K, epi=epi)
    finally:
        _lib.call("mlic_set_kernel_option", b"x4_halo", -1)
        _lib.call("mlic_set_kernel_option", b"x4_splitk", -1)
    for (y, ref) in res.values():
        check(y, ref)
    assert torch.equal(res[(0, 1)][0], res[(0, 0)][0])  # no split: halo == per-tap, bit for bit
    tiles = -(-cout // 256) * -(-W // 32) * -(-H // 8)
    if tiles > 48:  # split-K never applies (conv_x4.hip x4_splitk): forced on changes nothing
        assert torch.equal(res[(1, 1)][0], res[(0, 1)][0])


def _conv_raw(impl, x, w, b, epi):
    from mlic_amd import _lib
    B, Cin, H, W = x.shape
    y = torch.full((B, w.shape[0], H, W), float("nan"), device=x.device)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("mlic_conv_run", C.c_void_p(st), impl, C.c_void_p(x.data_ptr()), C.c_void_p(w.data_ptr()),
              C.c_void_p(b.data_ptr()), C.c_void_p(y.data_ptr()), B, Cin, w.shape[0], H, W, 1, 1, epi, None, None)
    torch.cuda.synchronize()
    return y


@pytest.mark.parametrize("shape", [
    (2, 640, 224, 17, 30),   # LRP point conv, 224-row tile
    (2, 960, 320, 17, 30),   # entropy-parameters GEMM, 2 Cout tiles
    (1, 100, 200, 9, 33),    # Cin 100: the last chunk's channels 96..99 real, the rest zeros
    (1, 70, 64, 5, 7),       # Cin 70: one 16-channel group ragged, one all zeros; 35 px: one ragged tile
    (2, 96, 96, 13, 37),     # 96-row tile
])
def test_x4_1x1_direct_vs_packed(shape):
    """1x1 layers: x4 builds the split B rows from the fp32 input itself (no packed copy); under SQUARE
    the pack kernel forms x^2 and the packed path runs.  Both multiply the same split operands in the
    same order, so conv(x, SQUARE) == conv(x * x) bit for bit, and both match float64."""
    B, cin, cout, H, W = shape
    g = torch.Generator().manual_seed(7)
    dev = torch.device("cuda")
    x = (torch.rand(B, cin, H, W, generator=g) - 0.5).to(dev)
    w = ((torch.rand(cout, cin, 1, 1, generator=g) - 0.5) / cin ** 0.5).to(dev)
    b = (torch.rand(cout, generator=g) - 0.5).to(dev)
    y_direct = _conv_raw(X4, x * x, w, b, 0)
    y_packed = _conv_raw(X4, x, w, b, SQUARE)
    assert torch.equal(y_direct, y_packed)
    check(y_direct, F.conv2d((x * x).double(), w.double(), b.double()).float())


@pytest.mark.parametrize("shape", [
    (2, 192, 192, 34, 60, 0),      # small-decoder g_a / h_a stride-2 dense conv
    (1, 192, 192, 33, 47, 1),      # odd input: the last output row / column reads the zero border
    (1, 320, 192, 17, 30, 1),      # 10 chunks, small grid: the split-K path
])
def test_x4_stride2(shape):
    B, cin, cout, H, W, epi = shape
    check(*run(X4, B, cin, cout, H, W, 3, stride=2, epi=epi))


def _fp16_operands(x, w):
    """The operands the reduced-precision x4 form multiplies: x rounded to fp16, w rounded to fp16
    after the layer's exact power-of-two prescale (max |w| * 2^e in [2^14, 2^15), split_weights)."""
    e = 14 - math.floor(math.log2(w.abs().max().item()))
    return x.half().double(), (w * 2.0 ** e).half().double() / 2.0 ** e


@pytest.mark.parametrize("shape", [
    (2, 192, 768, 24, 64, 3, SHUFFLE | GELU),   # g_s subpel conv (MLICPP_L): 3 chunks of 64 channels
    (1, 192, 768, 19, 45, 3, SHUFFLE),          # ragged pixel tiles at every edge
    (1, 96, 384, 16, 40, 3, SHUFFLE | GELU),    # MLICPP_S width: 96 channels = one zero-padded chunk pair
    (1, 100, 200, 9, 33, 3, RES),               # Cin not a multiple of 32, partial Cout tile, residual
    (1, 320, 64, 13, 37, 5, 0),                 # 5x5 with few tiles: the split-K path
    (1, 192, 192, 16, 40, 3, GELU),             # 192-row tile
])
def test_x4_fp16_operands(shape):
    """The reduced-precision synthesis form: fp16 x fp16 products with fp32 accumulation.
    Against float64 of the fp16-rounded operands it is exact to fp32 summation noise (2e-5), and
    against the fp32 conv it is within fp16 operand rounding (2e-3 of the output scale)."""
    from mlic_amd import _lib
    B, cin, cout, H, W, K, epi = shape
    y, ref = run(X4H, B, cin, cout, H, W, K, epi=epi)
    check(y, ref, rtol=2e-3)
    g = torch.Generator().manual_seed(0)  # run()'s operands, regenerated
    dev = torch.device("cuda")
    x = (torch.rand(B, cin, H, W, generator=g) - 0.5).to(dev)
    w = ((torch.rand(cout, cin, K, K, generator=g) - 0.5) / (cin * K * K) ** 0.5).to(dev)
    b = (torch.rand(cout, generator=g) - 0.5).to(dev)
    oshape = (B, cout // 4, 2 * H, 2 * W) if epi & SHUFFLE else (B, cout, H, W)
    res = (torch.rand(*oshape, generator=g) - 0.5).to(dev) if epi & RES else None
    xh, wh = _fp16_operands(x.double(), w.double())
    ref16 = reference(xh, wh, b.double(), 1, epi, res.double() if res is not None else None).float()
    check(y, ref16, rtol=2e-5)


def test_x4_auto_selection():
    """A g_s-shaped subpel conv whose grid fills the chip runs on x4 under automatic selection."""
    y, ref = run(AUTO, 2, 192, 768, 128, 192, 3, epi=SHUFFLE | GELU)
    check(y, ref)
    y2, _ = run(X4, 2, 192, 768, 128, 192, 3, epi=SHUFFLE | GELU)
    assert torch.equal(y, y2)


def test_auto_matches_selected_family():
    y, ref = run(AUTO, 2, 192, 192, 136, 240, 1, epi=GELU)
    check(y, ref)
    y2, _ = run(PW, 2, 192, 192, 136, 240, 1, epi=GELU)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("shape", [
    (2, 192, 64, 256, 1, 0),   # vectorised stride-1 path, 2 x 2 tiles
    (1, 64, 68, 120, 1, 1),    # latent grid: 24-row tiles (3 x 24 covers 68 rows), GELU
    (2, 192, 40, 100, 1, 1),   # W % 4 == 0, ragged tiles, GELU
    (1, 96, 37, 53, 1, 0),     # W % 4 != 0: generic path
    (2, 192, 64, 96, 2, 0),    # stride 2, vectorised path (W % 8 == 0)
    (2, 192, 68, 120, 2, 1),   # stride 2, ragged tile, GELU
    (1, 3, 65, 97, 2, 0),      # 3-channel stride-2 input conv, odd sizes
])
def test_depthwise(shape):
    from mlic_amd import _lib
    B, Cn, H, W, s, gelu = shape
    g = torch.Generator().manual_seed(1)
    dev = torch.device("cuda")
    x = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    w = (torch.rand(Cn, 1, 3, 3, generator=g) - 0.5).to(dev)
    b = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    y = torch.full((B, Cn, Ho, Wo), float("nan"), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("mlic_dw_run", C.c_void_p(st), C.c_void_p(x.data_ptr()), C.c_void_p(w.data_ptr()),
              C.c_void_p(b.data_ptr()), C.c_void_p(y.data_ptr()), B, Cn, H, W, s, gelu)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=s, padding=1, groups=Cn)
    if gelu:
        ref = F.gelu(ref)
    check(y, ref.float(), rtol=1e-6)


@pytest.mark.parametrize("B,Cn,H,W,gelu", [
    (2, 224, 32, 48, 0),    # Kodak-size latent: 12 float4 columns, 5 strips per wave, R = 17 (2 strips)
    (3, 64, 32, 48, 1),     # GELU
    (1, 32, 68, 64, 1),     # 16 columns: 4 strips per wave; 68 rows = 4 x 17
    (2, 96, 9, 16, 0),      # 4 columns, 16 strips per wave; R = 8 / 12 tails
    (1, 40, 1, 8, 1),       # a single row: both vertical taps out of the image
    (2, 128, 25, 60, 0),    # 15 columns: the last lane pair of each strip at the wave seam
])
def test_depthwise_strip_vs_tile(B, Cn, H, W, gelu):
    """The register-strip depthwise (narrow stride-1 planes) == the LDS-tile kernel, bit for bit (same
    fma order), and == float64 torch to 1e-6."""
    from mlic_amd import _lib
    g = torch.Generator().manual_seed(5)
    dev = torch.device("cuda")
    x = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    w = (torch.rand(Cn, 1, 3, 3, generator=g) - 0.5).to(dev)
    b = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    outs = {}
    for mode in (1, 0):
        y = torch.full((B, Cn, H, W), float("nan"), device=dev)
        _lib.call("mlic_set_kernel_option", b"dw_strip", mode)
        try:
            _lib.call("mlic_dw_run", C.c_void_p(st), C.c_void_p(x.data_ptr()), C.c_void_p(w.data_ptr()),
                      C.c_void_p(b.data_ptr()), C.c_void_p(y.data_ptr()), B, Cn, H, W, 1, gelu)
        finally:
            _lib.call("mlic_set_kernel_option", b"dw_strip", -1)
        outs[mode] = y
    assert torch.equal(outs[0], outs[1])
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1, groups=Cn)
    if gelu:
        ref = F.gelu(ref)
    check(outs[1], ref.float(), rtol=1e-6)


@pytest.mark.parametrize("B,Cn,H,W,epi", [
    (2, 192, 40, 100, 1),    # GELU; 100 columns = one 60-column segment + a ragged 40
    (1, 192, 17, 61, 0),     # odd width: refused (the model runs it unfused)
    (2, 192, 68, 120, 1 | 64),  # latent grid, GELU + residual
    (1, 128, 24, 30, 0),     # Cin 128, one ragged segment
    (3, 192, 20, 96, 64),    # residual only
    (2, 160, 9, 64, 1),      # MLICPP_M width
    (2, 96, 33, 70, 1 | 64), # MLICPP_S width
    (2, 48, 16, 160, 1 | 64),  # the small-decoder model's g_s width (3 k-steps: odd count)
    (1, 192, 1, 34, 1),      # a single row: both vertical taps out of the image
    (2, 192, 13, 120, 1 | 64),  # two exact segments, ragged row block
    (1, 192, 6, 62, 0),      # one segment + one pixel pair
    (1, 96, 3, 2, 1),        # a single pair: both halo pairs out of the image
    (1, 192, 5, 960, 1),     # full-resolution width
    (2, 128, 8, 184, 64),    # Cin 128, ragged last segment (4 pairs)
    # Cin = Cout in 96..192 (the default register-row form, conv_dwpw3.hip)
    (2, 192, 98, 480, 1 | 64),  # several 6 x 32 tiles per workgroup, ragged row block (98 = 16 x 6 + 2)
    (1, 160, 100, 320, 1),   # N = 160, 5 consumer waves
    (2, 96, 40, 228, 0),     # N = 96, ragged last column tile (228 = 7 x 32 + 4)
])
def test_dwpw_fused(B, Cn, H, W, epi):
    """Fused depthwise 3x3 + pointwise 1x1 (conv_dwpw.hip) == depthwise kernel then the resident-weight
    pointwise kernel, bit for bit (same depthwise order, same MFMA k order), and within the split-fp16
    tolerance of a float64 torch reference (DepthWiseConv, modules/layers/conv.py:22-32)."""
    _dwpw_case(B, Cn, Cn, H, W, epi)


@pytest.mark.parametrize("form", [0, 1, 2])
@pytest.mark.parametrize("B,Cn,H,W,epi", [
    (2, 192, 68, 120, 1 | 64), (3, 192, 20, 96, 64), (2, 192, 98, 480, 1 | 64), (1, 160, 100, 320, 1),
    (2, 96, 40, 228, 0), (2, 128, 8, 184, 64), (1, 192, 5, 960, 1), (2, 192, 40, 100, 1),
    (1, 96, 33, 62, 1 | 64), (2, 160, 9, 130, 1), (1, 128, 70, 64, 1 | 64)])
def test_dwpw2_fused(B, Cn, H, W, epi, form):
    """The fused Cin = Cout forms (mlic_set_kernel_option("dwpw2", form)): 0 = dwpw_kernel (conv_dwpw.hip,
    one wave per SIMD; its Cin = Cout instantiations are in the A/B library only since round 6), 1 = the
    row-pipelined LDS form (ab/conv_dwpw2.hip, A/B-only library), 2 = the
    register-row form (conv_dwpw3.hip, the default; 64-pixel strips: ragged, narrower-than-a-strip and
    exact-multiple widths): the same bits as depthwise + resident pointwise.  (2, 192, 68, 120, GELU +
    residual) and (3, 192, 20, 96, residual) are the shapes on which form 1's masked-residual builds
    returned wrong rows."""
    from mlic_amd import _lib
    if form in (0, 1) and not _lib.ab_families():
        pytest.skip("forms 0 / 1 are A/B-only instantiations for Cin = Cout (make AB=1)")
    _lib.call("mlic_set_kernel_option", b"dwpw2", form)
    try:
        _dwpw_case(B, Cn, Cn, H, W, epi)
    finally:
        _lib.call("mlic_set_kernel_option", b"dwpw2", -1)


@pytest.mark.parametrize("B,Cn,H,W,epi", [
    (1, 192, 136, 128, GDN | SQUARE | RES), (2, 192, 130, 130, IGDN | SQUARE | RES), (1, 160, 128, 200, GDN | SQUARE),
    (1, 128, 200, 100, IGDN | SQUARE), (2, 96, 64, 300, GDN | SQUARE | RES),
    (2, 192, 136, 240, GELU), (1, 192, 130, 140, 0), (1, 160, 128, 130, GELU | RES)])
def test_pw3_gdn(B, Cn, H, W, epi):
    """The full-resolution GDN / IGDN 1x1 on the register-row kernel's pointwise form (conv_dwpw3.hip, PW):
    bit for bit pw_resident's (x^2 split, MFMA order, x * rsqrt / sqrt epilogue, residual last), and
    within tolerance of the float64 reference."""
    from mlic_amd import _lib
    try:
        _lib.call("mlic_set_kernel_option", b"pw3", 0)
        y0, ref = run(PW, B, Cn, Cn, H, W, 1, epi=epi, seed=3)
        _lib.call("mlic_set_kernel_option", b"pw3", 2)  # (2: at every grid; the default takes >= 256 K px)
        y1, _ = run(PW, B, Cn, Cn, H, W, 1, epi=epi, seed=3)
    finally:
        _lib.call("mlic_set_kernel_option", b"pw3", -1)
    check(y1, ref)
    assert torch.equal(y0, y1)


# the latent-resolution dwsep convs with Cin != Cout: the LRP's 224 -> 128 GELU and its 128 -> 32 head
# (0.5 tanh, checkerboard mask, residual; quantization.py:30-45), the channel context's 192 -> 128 GELU
@pytest.mark.parametrize("B,Cin,Cout,H,W,epi", [
    (2, 224, 128, 68, 120, 1), (1, 224, 128, 17, 30, 1),
    (2, 128, 32, 68, 120, 8 | 16 | 64), (2, 128, 32, 17, 30, 8 | 32 | 64), (1, 128, 32, 9, 14, 8 | 16 | 64),
    (2, 192, 128, 68, 120, 1), (1, 192, 128, 16, 24, 1)])
def test_dwpw_fused_latent(B, Cin, Cout, H, W, epi):
    _dwpw_case(B, Cin, Cout, H, W, epi)


def _dwpw_case(B, Cn, Cout, H, W, epi):
    from mlic_amd import _lib
    TANH, MASK_A, MASK_N, EPI_RES = 8, 16, 32, 64
    g = torch.Generator().manual_seed(5)
    dev = torch.device("cuda")
    x = (torch.rand(B, Cn, H, W, generator=g) - 0.5).to(dev)
    dw = ((torch.rand(Cn, 1, 3, 3, generator=g) - 0.5) * 0.6).to(dev)
    db = (torch.rand(Cn, generator=g) - 0.5).to(dev)
    w = ((torch.rand(Cout, Cn, 1, 1, generator=g) - 0.5) * 0.2).to(dev)
    b = (torch.rand(Cout, generator=g) - 0.5).to(dev)
    res = (torch.rand(B, Cout, H, W, generator=g) - 0.5).to(dev)
    st = torch.cuda.current_stream().cuda_stream
    y = torch.full((B, Cout, H, W), float("nan"), device=dev)
    args = (C.c_void_p(st), C.c_void_p(x.data_ptr()), C.c_void_p(dw.data_ptr()), C.c_void_p(db.data_ptr()),
            C.c_void_p(w.data_ptr()), C.c_void_p(b.data_ptr()), C.c_void_p(y.data_ptr()), B, Cn, Cout, H, W, epi,
            C.c_void_p(res.data_ptr()))
    if W % 2:  # a lane's pixel pair must be inside the row or outside it: the model runs these unfused
        with pytest.raises(_lib.MlicError):
            _lib.call("mlic_dwpw_run", *args)
        return
    _lib.call("mlic_dwpw_run", *args)
    t = torch.full((B, Cn, H, W), float("nan"), device=dev)
    _lib.call("mlic_dw_run", C.c_void_p(st), C.c_void_p(x.data_ptr()), C.c_void_p(dw.data_ptr()),
              C.c_void_p(db.data_ptr()), C.c_void_p(t.data_ptr()), B, Cn, H, W, 1, 0)
    y2 = torch.full((B, Cout, H, W), float("nan"), device=dev)
    _lib.call("mlic_conv_run", C.c_void_p(st), 3, C.c_void_p(t.data_ptr()), C.c_void_p(w.data_ptr()),
              C.c_void_p(b.data_ptr()), C.c_void_p(y2.data_ptr()), B, Cn, Cout, H, W, 1, 1, epi, None,
              C.c_void_p(res.data_ptr()))
    assert torch.equal(y, y2)
    ref = F.conv2d(F.conv2d(x.double(), dw.double(), db.double(), padding=1, groups=Cn), w.double(), b.double())
    if epi & 1:
        ref = F.gelu(ref)
    if epi & TANH:
        ref = 0.5 * torch.tanh(ref)
    if epi & (MASK_A | MASK_N):  # checkerboard: anchor cells have (h + w) odd
        hh = torch.arange(H, device=dev).view(-1, 1)
        ww = torch.arange(W, device=dev).view(1, -1)
        anchor = ((hh + ww) % 2) == 1
        ref = ref * (anchor if epi & MASK_A else ~anchor).to(ref.dtype)
    if epi & EPI_RES:
        ref = ref + res.double()
    check(y, ref.float(), rtol=1e-6)


def test_gelu_accuracy():
    """The conv / depthwise epilogues' device GELU (common.h gelu_epi: torch's 0.5 x (1 + erf(x /
    sqrt 2)) on the library erff) on a dense grid over [-12, 12]: its error vs the exact GELU (float64)
    stays within 6 ulp of max(|x|, 2^-10), as torch's own fp32 GELU does (5.1).  (The chain kernel's
    branch-free gelu_erf is pinned through the chain-vs-oracle parity tests.)  Driven through the
    depthwise kernel with the centre tap 1 and zero bias, so y = gelu(x) exactly."""
    from mlic_amd import _lib
    dev = torch.device("cuda")
    n = 1 << 20
    xs = torch.linspace(-12.0, 12.0, n, dtype=torch.float32)
    H, W = 1024, 1024
    x = xs.reshape(1, 1, H, W).to(dev)
    w = torch.zeros(1, 1, 3, 3, device=dev)
    w[0, 0, 1, 1] = 1.0
    b = torch.zeros(1, device=dev)
    y = torch.full_like(x, float("nan"))
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("mlic_dw_run", C.c_void_p(st), C.c_void_p(x.data_ptr()), C.c_void_p(w.data_ptr()),
              C.c_void_p(b.data_ptr()), C.c_void_p(y.data_ptr()), 1, 1, H, W, 1, 1)
    torch.cuda.synchronize()
    xd = xs.double()
    exact = 0.5 * xd * torch.special.erfc(-xd / math.sqrt(2.0))
    scale = torch.clamp(xs.abs(), min=2.0 ** -10)
    ulp = (torch.nextafter(scale, torch.tensor(float("inf"))) - scale).double()
    dev_ulps = ((y.cpu().reshape(-1).double() - exact).abs() / ulp).max().item()
    torch_ulps = ((F.gelu(xs).double() - exact).abs() / ulp).max().item()
    assert dev_ulps <= 6.0, (dev_ulps, torch_ulps)


@pytest.mark.parametrize("ch,H,W,B", [(32, 24, 40, 2), (64, 13, 21, 1), (32, 68, 120, 1)])
def test_local_attention_kernels(ch, H, W, B):
    """Both LocalContext attention kernels vs a float64 torch restatement of context.py:75-107."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import mlic_ref_cpu as ref
    from mlic_amd import _lib, synthetic
    g = torch.Generator().manual_seed(3)
    dev = torch.device("cuda")
    heads, hd, L = 2, ch // 2, H * W
    qkv = (torch.randn(B, 3 * ch, H, W, generator=g) * 2).to(dev)
    table = torch.randn(81, 2, generator=g).to(dev)
    index = torch.from_numpy(synthetic.relative_position_index(5)).reshape(-1).to(torch.int32).to(dev)
    scale = hd ** -0.5
    x = qkv.double()
    wins = F.unfold(x, kernel_size=5, padding=2).permute(0, 2, 1).reshape(B, L, 3, ch, 25).permute(2, 0, 1, 3, 4)

    def heads_split(t):  # channel c = d * heads + h
        return t.reshape(B, L, hd, heads, 25).permute(0, 1, 3, 4, 2)
    q, k, v = heads_split(wins[0]) * scale, heads_split(wins[1]), heads_split(wins[2])
    bias = table.double()[index.long()].view(25, 25, 2).permute(2, 0, 1)
    mask = ref.local_attn_mask(H, W, 5).double().to(dev)
    attn = torch.softmax(q @ k.transpose(-2, -1) + bias[None, None] + mask[None, :, None], dim=-1)
    expect = (attn @ v).permute(0, 2, 4, 3, 1).reshape(B, ch * 25, H, W).float()  # row (h * hd + d) * 25 + i
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    impls = (0, 1) if _lib.ab_families() else (1,)  # 0: the A/B-only VALU kernel
    for impl in impls:
        out = torch.full((B, 25 * ch, H, W), float("nan"), device=dev)
        _lib.call("mlic_local_attn_run", C.c_void_p(st), impl, C.c_void_p(qkv.data_ptr()),
                  C.c_void_p(table.data_ptr()), C.c_void_p(index.data_ptr()), C.c_void_p(out.data_ptr()),
                  ch, H, W, B, float(scale))
        outs.append(out)
    report = []
    for impl, out in zip(impls, outs):
        d = (out - expect).abs()
        k = int(d.argmax())
        idx = [int(v) for v in torch.unravel_index(torch.tensor(k), d.shape)]
        report.append(f"impl{impl}: max {d.max().item():.3e} at {idx} (ref {expect.flatten()[k].item():.4f})")
    print("; ".join(report))
    for out in outs:
        assert torch.isfinite(out).all()
        # softmax of logits with |q.k| up to ~40 amplifies fp32 rounding of the scores; the bound is
        # on the mean error plus a looser max (the model-level parity tests hold bpp / PSNR)
        d = (out - expect).abs()
        assert d.mean().item() <= 1e-5 * expect.abs().mean().item() + 1e-7, report
        assert d.max().item() <= 1e-3 * expect.abs().max().item(), report


@pytest.mark.parametrize("H,W,B", [(24, 40, 2), (68, 120, 1), (13, 21, 1)])
def test_local_attention_packed(H, W, B):
    """The packed-output attention (dim 32) against the float64 torch restatement of
    context.py:75-107: hi + lo of the packed layout [B][cell][pos][64] re-ordered to row
    (head*16 + d)*25 + cell, with the tolerances of test_local_attention_kernels."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import mlic_ref_cpu as ref
    from mlic_amd import _lib, synthetic
    g = torch.Generator().manual_seed(5)
    dev = torch.device("cuda")
    ch, heads, hd, L = 32, 2, 16, H * W
    qkv = (torch.randn(B, 3 * ch, H, W, generator=g) * 2).to(dev)
    table = torch.randn(81, 2, generator=g).to(dev)
    index = torch.from_numpy(synthetic.relative_position_index(5)).reshape(-1).to(torch.int32).to(dev)
    scale = hd ** -0.5
    x = qkv.double()
    wins = F.unfold(x, kernel_size=5, padding=2).permute(0, 2, 1).reshape(B, L, 3, ch, 25).permute(2, 0, 1, 3, 4)

    def heads_split(t):  # channel c = d * heads + h
        return t.reshape(B, L, hd, heads, 25).permute(0, 1, 3, 4, 2)
    q, k, v = heads_split(wins[0]) * scale, heads_split(wins[1]), heads_split(wins[2])
    bias = table.double()[index.long()].view(25, 25, 2).permute(2, 0, 1)
    mask = ref.local_attn_mask(H, W, 5).double().to(dev)
    attn = torch.softmax(q @ k.transpose(-2, -1) + bias[None, None] + mask[None, :, None], dim=-1)
    expect = (attn @ v).permute(0, 2, 4, 3, 1).reshape(B, ch * 25, H, W).float()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    npos = (H * W + 31) // 32 * 32
    out = torch.zeros(B, 25, npos, 64, dtype=torch.float16, device=dev)
    _lib.call("mlic_local_attn_packed_run", st, C.c_void_p(qkv.data_ptr()), C.c_void_p(table.data_ptr()),
              C.c_void_p(index.data_ptr()), C.c_void_p(out.data_ptr()), H, W, B, float(scale))
    got = out[..., :32].float() + out[..., 32:].float()                    # [B, cell, pos, channel]
    got = got[:, :, :L].permute(0, 3, 1, 2).reshape(B, 25 * ch, H, W)   # row channel*25 + cell
    assert torch.isfinite(got).all()
    d = (got - expect).abs()
    assert d.mean().item() <= 1e-5 * expect.abs().mean().item() + 1e-7, d.mean().item()
    assert d.max().item() <= 1e-3 * expect.abs().max().item(), d.max().item()


@pytest.mark.parametrize("H,W,B", [(24, 40, 2), (68, 120, 1), (14, 22, 1)])
def test_local_attention_packed_half(H, W, B):
    """Round 6: the packed attention over one checkerboard phase's query pixels (the slice loop's
    LocalContext runs it on the non-anchor half): bit-identical to the whole-grid kernel's output at those
    pixels, written at their squeezed positions y * W / 2 + x / 2."""
    from mlic_amd import _lib, synthetic
    g = torch.Generator().manual_seed(6)
    dev = torch.device("cuda")
    qkv = (torch.randn(B, 96, H, W, generator=g) * 2).to(dev)
    table = torch.randn(81, 2, generator=g).to(dev)
    index = torch.from_numpy(synthetic.relative_position_index(5)).reshape(-1).to(torch.int32).to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    npos = (H * W + 31) // 32 * 32
    full = torch.zeros(B, 25, npos, 64, dtype=torch.int16, device=dev)
    _lib.call("mlic_local_attn_packed_run", st, C.c_void_p(qkv.data_ptr()), C.c_void_p(table.data_ptr()),
              C.c_void_p(index.data_ptr()), C.c_void_p(full.data_ptr()), H, W, B, 0.25)
    yy, xx = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    for ckbd in (1, 2):
        nq = (H * W // 2 + 31) // 32 * 32
        half = torch.zeros(B, 25, nq, 64, dtype=torch.int16, device=dev)
        _lib.call("mlic_local_attn_packed_half_run", st, C.c_void_p(qkv.data_ptr()), C.c_void_p(table.data_ptr()),
                  C.c_void_p(index.data_ptr()), C.c_void_p(half.data_ptr()), H, W, B, 0.25, ckbd)
        sel = (((yy + xx) % 2) == (1 if ckbd == 1 else 0)).reshape(-1)   # anchors: (y + x) odd
        want = full[:, :, :H * W][:, :, sel.to(dev)]
        assert torch.equal(half[:, :, :H * W // 2], want), ckbd


# split-fp16 operand range (conv_f16x3.hip header): tiny weights (the per-row power-of-two prescale keeps
# their lo halves normal) and activations up to 1e3, every split family, against float64
@pytest.mark.parametrize("impl,Cin,Cout,H,W,K", [(X3V2, 192, 320, 24, 40, 1), (X3V2, 96, 96, 20, 36, 3),
                                                 (PW, 192, 192, 36, 60, 1), (X4, 192, 768, 16, 64, 3),
                                                 (HALO, 96, 96, 24, 64, 5)])
@pytest.mark.parametrize("wmul,xmul", [(1e-3, 2e3), (1e-4, 1.0), (3e-5, 5e2)])
def test_split_operand_range(impl, Cin, Cout, H, W, K, wmul, xmul):
    needs_ab(impl)
    y, ref = run(impl, 2, Cin, Cout, H, W, K, wmul=wmul, xmul=xmul)
    check(y, ref, rtol=2e-5)
