"""CPU-side checks of libmlic_hip.so: it loads, exports the whole C ABI, and its host entropy
coder / CDF quantizer match the restated compressai behaviour and the reference fixtures."""
import ctypes as C
import os
import re

import numpy as np
import pytest
import torch

import rans_ref
from mlic_amd import _lib, entropy, synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "mlic_hip.h")).read()
    names = sorted(set(re.findall(r"\b(mlic_[a-z0-9_]+)\s*\(", hdr)))
    assert len(names) >= 15
    lib = _lib.lib()
    for n in names:
        assert hasattr(lib, n), n
    assert lib.mlic_version().startswith(b"mlic_hip")


def test_null_handle_is_an_error_not_a_crash():
    import ctypes as C
    hs = [C.c_double() for _ in range(3)]
    with pytest.raises(_lib.MlicError, match="null mlic_model handle"):
        _lib.call("mlic_host_stats", None, *[C.byref(v) for v in hs], 1)
    with pytest.raises(_lib.MlicError, match="null mlic_model handle"):
        _lib.call("mlic_set_lanes", None, 2)


def test_conv_choice_is_batch_independent():
    """The kernel family of every conv shape the models run (and a sweep around them) is the same for
    any batch size: families round differently, and a stream coded in a batch must decode alone."""
    shapes = []
    for H, W in ((68, 120), (32, 48), (136, 240), (272, 480), (544, 960), (17, 30), (8, 12), (64, 64)):
        for Cin, Cout, K in ((192, 192, 1), (128, 128, 1), (96, 96, 1), (160, 160, 1), (640, 6400, 1),
                             (480, 640, 1), (496, 224, 1), (224, 128, 1), (128, 32, 1), (32, 96, 1),
                             (192, 768, 3), (192, 192, 3), (320, 320, 5), (256, 64, 5), (3, 192, 1),
                             (192, 12, 3), (320, 640, 3)):
            for stride in ((1, 2) if K != 5 else (1,)):
                shapes.append((Cin, Cout, H, W, K, stride))
    impl = C.c_int()
    for Cin, Cout, H, W, K, stride in shapes:
        got = set()
        for B in (1, 2, 3, 8, 16, 64):
            _lib.call("mlic_conv_choice", B, Cin, Cout, H, W, K, stride, 0, C.byref(impl))
            got.add(impl.value)
        assert len(got) == 1, (Cin, Cout, H, W, K, stride, got)


def test_gaussian_tables_match_reference_update(golden):
    g = golden("scale_table.npz")
    cdf, length, offset, table = entropy.gaussian_tables(entropy.get_scale_table())
    assert torch.equal(table, torch.from_numpy(g["table"]))
    assert np.array_equal(cdf.numpy(), g["quantized_cdf"])
    assert np.array_equal(length.numpy(), g["cdf_length"])
    assert np.array_equal(offset.numpy(), g["offset"])


def _eb_params(sd):
    return {k.split(".", 1)[1]: v for k, v in sd.items() if k.startswith("entropy_bottleneck.")
            and (".quantiles" in k or "._" in k) and not k.endswith(("_offset", "_quantized_cdf", "_cdf_length"))}


def test_bottleneck_tables_match_reference_update(golden):
    g = golden("eb_cdf_L.npz")
    sd = synthetic.synth_state_dict("MLICPP_L", 0)
    cdf, length, offset = entropy.bottleneck_tables(_eb_params(sd))
    assert np.array_equal(cdf.numpy(), g["quantized_cdf"])
    assert np.array_equal(length.numpy(), g["cdf_length"])
    assert np.array_equal(offset.numpy(), g["offset"])


def test_bottleneck_tables_every_weight_set_and_form_diff(golden):
    """EntropyBottleneck.update() (mlicpp.py:470-475 -> compressai 1.2.6) on every fixture weight set:
    the product's z CDF tables equal the reference's, entry for entry.  Also counts how many quantised
    CDF entries the compressai-1.1 sign-trick pmf would change -- the entries where a coder built on the
    wrong form would write z streams a reference decoder cannot read (recorded in $MLIC_PARITY_OUT)."""
    import hashlib
    import json
    g = golden("eb_cdf_sets.npz")
    tags = sorted({k.split(".")[0] for k in g.files})
    assert len(tags) >= 10
    rec = {}
    for tag in tags:
        name, rate = (tag.rsplit("_r", 1)[0], int(tag.rsplit("_r", 1)[1])) if "_r" in tag[-3:] else (tag, None)
        sd = synthetic.synth_state_dict(name, 0, rate=rate)
        h = hashlib.sha256()
        for k in sorted(sd):
            h.update(k.encode())
            h.update(sd[k].contiguous().numpy().tobytes())
        assert h.hexdigest() == str(g[f"{tag}.sd_sha"]), tag
        p = _eb_params(sd)
        cdf, length, offset = entropy.bottleneck_tables(p)
        assert np.array_equal(cdf.numpy(), g[f"{tag}.quantized_cdf"]), tag
        assert np.array_equal(length.numpy(), g[f"{tag}.cdf_length"]), tag
        assert np.array_equal(offset.numpy(), g[f"{tag}.offset"]), tag
        old, _, _ = entropy.bottleneck_tables(p, sign_trick=True)
        diff = old.numpy() != cdf.numpy()
        rec[tag] = {"entries": int(cdf.numel()), "sign_trick_entries_differing": int(diff.sum()),
                    "channels_differing": int(diff.any(axis=1).sum()), "channels": int(cdf.shape[0])}
    out = os.environ.get("MLIC_PARITY_OUT")
    if out:
        old_rec = json.load(open(out)) if os.path.exists(out) else {}
        old_rec["eb_cdf_form_diff"] = rec
        with open(out, "w") as f:
            json.dump(old_rec, f, indent=1, sort_keys=True)
    print(json.dumps(rec))


def _gc_tables(golden):
    g = golden("scale_table.npz")
    return g["quantized_cdf"], g["cdf_length"], g["offset"]


def test_rans_roundtrip_reference_streams(golden):
    cdf, length, offset = _gc_tables(golden)
    f = golden("forward_MLICPP_L_128x192.npz")
    sym, idx = f["y_symbols"], f["y_indexes"]
    data = entropy.rans_encode(sym, idx, cdf, length, offset)
    assert len(data) % 4 == 0
    back = entropy.rans_decode(data, idx, cdf, length, offset)
    assert np.array_equal(back, sym)
    # bytes identical to the pure-Python restatement of compressai's coder
    n = 20000
    ref = rans_ref.encode(sym[:n].tolist(), idx[:n].tolist(), cdf.tolist(), length.tolist(), offset.tolist())
    assert entropy.rans_encode(sym[:n], idx[:n], cdf, length, offset) == ref


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_rans_bypass_and_extremes(golden, seed):
    cdf, length, offset = _gc_tables(golden)
    r = np.random.default_rng(seed)
    n = 5000
    idx = r.integers(0, 64, n).astype(np.int32)
    sym = (r.standard_normal(n) * r.choice([0.5, 3, 40, 3000], n)).astype(np.int32)
    sym[:8] = [0, -1, 1, 2 ** 20, -(2 ** 20), 2 ** 30, -(2 ** 30), 123456]
    data = entropy.rans_encode(sym, idx, cdf, length, offset)
    assert np.array_equal(entropy.rans_decode(data, idx, cdf, length, offset), sym)
    ref = rans_ref.encode(sym.tolist(), idx.tolist(), cdf.tolist(), length.tolist(), offset.tolist())
    assert data == ref


def _decode_narrow(data, idx8, nparts, cdf, length, offset):
    cdf_, length_, offset_ = (np.ascontiguousarray(np.asarray(v), dtype=np.int32) for v in (cdf, length, offset))
    out = np.zeros(idx8.size, np.int32)
    widened = C.c_int(-1)
    _lib.call("mlic_rans_decode_narrow", data, len(data), idx8.ctypes.data, idx8.size, nparts, cdf_.ctypes.data,
              length_.ctypes.data, offset_.ctypes.data, cdf_.shape[0], cdf_.shape[1], out.ctypes.data,
              C.byref(widened))
    return out, widened.value


@pytest.mark.parametrize("limit", [0, 40, 3])
def test_rans_narrow_decode_fallback(golden, limit):
    """The decompress path's narrow decode: each phase is decoded into int16 and, when a value
    leaves the narrow range, the decoder resets to the phase's start and decodes it again into int32
    (PhaseDecoder::run -> rans_decode_piece).  The narrow range is lowered with the "narrow_limit" knob so
    that the fallback runs here: the symbols must come back exactly, the pieces that widen are exactly the
    ones holding an out-of-range value, and the stream is consumed in step (later pieces decode right)."""
    cdf, length, offset = _gc_tables(golden)
    r = np.random.default_rng(11)
    nparts, npiece = 20, 750
    idx8 = r.integers(0, 64, nparts * npiece).astype(np.uint8)
    sym = (r.standard_normal(nparts * npiece) * 4).astype(np.int32)
    sym[3 * npiece + 7] = 70000            # beyond int16: piece 3 must widen at every limit
    sym[8 * npiece + 100] = -40000         # piece 8 too
    sym[12 * npiece + 5] = 41              # beyond the limit of 40 only
    data = entropy.rans_encode(sym, idx8.astype(np.int32), cdf, length, offset)
    try:
        _lib.call("mlic_set_kernel_option", b"narrow_limit", limit)
        back, widened = _decode_narrow(data, idx8, nparts, cdf, length, offset)
    finally:
        _lib.call("mlic_set_kernel_option", b"narrow_limit", 0)
    assert np.array_equal(back, sym)
    lim = 32767 if limit <= 0 else limit
    want = sum(1 for k in range(nparts) if np.any((sym[k * npiece:(k + 1) * npiece] > lim) |
                                                  (sym[k * npiece:(k + 1) * npiece] < -lim - 1)))
    assert widened == want and widened >= 2
    # the plain int32 decoder agrees on the same stream
    assert np.array_equal(entropy.rans_decode(data, idx8.astype(np.int32), cdf, length, offset), sym)


def test_rans_empty_stream(golden):
    cdf, length, offset = _gc_tables(golden)
    data = entropy.rans_encode(np.zeros(0, np.int32), np.zeros(0, np.int32), cdf, length, offset)
    assert len(data) == 8
    assert entropy.rans_decode(data, np.zeros(0, np.int32), cdf, length, offset).size == 0


def test_pmf_to_quantized_cdf_properties():
    r = np.random.default_rng(3)
    for n in (2, 5, 37, 300):
        p = r.dirichlet(np.ones(n) * 0.3).astype(np.float32)
        p[r.integers(0, n)] = 0.0  # zero-probability symbols must still get frequency >= 1
        c = entropy.pmf_to_quantized_cdf(p)
        assert c[0] == 0 and c[-1] == 1 << 16
        assert np.all(np.diff(c) >= 1)


def test_conv_choice_pins_the_measured_selection():
    """The kernel family per layer shape that the A/B measurements chose; a
    regression here changes speed (and, as families round differently, the exact bits)."""
    F32, X3, X3V2, PW, NARROW, SMALLCIN, HALO, X4 = range(8)
    impl = C.c_int()

    def choice(Cin, Cout, H, W, K, stride=1, B=8, epi=0):
        _lib.call("mlic_conv_choice", B, Cin, Cout, H, W, K, stride, epi, C.byref(impl))
        return impl.value

    assert choice(192, 768, 272, 480, 3) == X4            # g_s subpel convs
    assert choice(320, 1280, 8, 12, 3) == X4              # h_s subpel at the Kodak z grid (split-K)
    assert choice(192, 192, 544, 960, 1) == PW            # full-resolution point convs
    assert choice(224, 128, 32, 48, 1, epi=1) == PW       # Kodak-size LRP.2 (GELU): resident from 1 K px
    assert choice(224, 128, 17, 30, 1, epi=1) != PW       # below 1 K px/image
    assert choice(288, 288, 68, 120, 1) == X4             # context q/k/v (Cin <= 352)
    assert choice(640, 224, 68, 120, 1, epi=1) == X4      # 1080p LRP point conv: 1.07x x3v2
    assert choice(640, 224, 32, 48, 1, epi=1) == X4       # Kodak LRP: 1.3x
    assert choice(160, 96, 68, 120, 1) == X3V2            # narrow latent 1x1s without a resident form
    assert choice(640, 6400, 68, 120, 1) == X4            # hoisted EntropyParameters GEMM
    assert choice(288, 96, 68, 120, 5) == X4              # 5x5 reprojections
    assert choice(192, 192, 544, 960, 3, stride=2) == X4  # small-decoder dense strided conv
    assert choice(96, 128, 68, 120, 3) == X4              # small-decoder channel context: 1.4x x3v2
    assert choice(288, 96, 68, 120, 3, epi=1) == X4       # 1.5x
    assert choice(3, 192, 1088, 1920, 3, stride=2) == SMALLCIN
    assert choice(3, 192, 1088, 1920, 1, stride=2) == SMALLCIN
    assert choice(192, 12, 544, 960, 3) == NARROW
    assert choice(48, 48, 1088, 1920, 1) == PW            # small-decoder g_s width


@pytest.mark.parametrize("vbr", [False, True])
def test_file_bytes_is_the_written_file_size(vbr):
    """bench.py's bpp_file counts the whole file the harness writes (utils/utils.py:71-83)."""
    import io
    from mlic_amd import bitstream
    y, z = b"\x01" * 37, b"\x02" * 5
    buf = io.BytesIO()
    n = bitstream.write_stream(buf, 120, 200, (2, 4), [[y], [z]], level=3 if vbr else None)
    assert n == len(buf.getvalue()) == bitstream.file_bytes(len(y), len(z), vbr=vbr)
    buf.seek(0)
    hdr, strings, shape = bitstream.read_stream(buf, vbr=vbr)
    assert strings == [[y], [z]] and shape == (2, 4) and hdr[:2] == (120, 200)


def test_build_record_matches_tree():
    """The in-tree library carries a record of the sources it was built from (mlic_amd/build.py); it
    matches the tree, and the recorded library digest is the library's."""
    import hashlib
    import json
    from mlic_amd import build
    rec = json.load(open(build.RECORD))
    assert rec["sources_sha256"] == build.source_digest()
    assert rec["library_sha256"] == hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()
    assert rec["target"] == "gfx950"
