// C ABI of libmlic_hip.so (include/mlic_hip.h): status codes, thread-local error text.
#include "../../include/mlic_hip.h"

#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "model.h"

using namespace mlic;

struct mlic_model {
  Model* impl;
};

static thread_local std::string g_err;

template <class F>
static int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "mlic: unknown error";
  }
  return 1;
}

// Every entry point that takes a handle goes through here: a null handle is an error, not a crash.
static Model& impl(mlic_model* m) {
  MLIC_CHECK(m != nullptr && m->impl != nullptr, "null mlic_model handle");
  return *m->impl;
}

static CdfTables make_tables(const int32_t* cdf, const int32_t* len, const int32_t* off, int n, int stride) {
  CdfTables t;
  t.n = n;
  t.stride = stride;
  t.cdf.assign(cdf, cdf + (size_t)n * stride);
  t.length.assign(len, len + n);
  t.offset.assign(off, off + n);
  for (int i = 0; i < n; ++i)
    MLIC_CHECK(t.length[i] >= 3 && t.length[i] <= stride, "cdf length out of range");
  t.prepare();
  return t;
}

extern "C" {

const char* mlic_last_error(void) { return g_err.c_str(); }
const char* mlic_version(void) { return "mlic_hip 0.1 gfx950"; }

int mlic_create(const char* model_name, int n, const char* const* names, const float* const* ptrs,
                const int64_t* shapes, const int* ndims, void* stream, mlic_model** out) {
  return guard([&] {
    MLIC_CHECK(out != nullptr, "null out");
    auto* m = new mlic_model{nullptr};
    try {
      m->impl = new Model(model_name, n, names, ptrs, shapes, ndims, (hipStream_t)stream);
      if (const char* e = std::getenv("MLIC_LANES")) m->impl->set_lanes(std::atoi(e));
      if (const char* e = std::getenv("MLIC_PRECISION")) m->impl->set_precision(std::atoi(e));
      if (const char* e = std::getenv("MLIC_SYNTH_FP16")) m->impl->set_synthesis_precision(std::atoi(e) == 1 ? 1 : 0);
      if (const char* e = std::getenv("MLIC_POISON")) m->impl->set_poison(std::atoi(e) != 0);
    } catch (...) {
      delete m;
      throw;
    }
    *out = m;
  });
}

int mlic_destroy(mlic_model* m) {
  return guard([&] {
    if (!m) return;
    delete m->impl;
    delete m;
  });
}

int mlic_forward(mlic_model* m, void* stream, const float* x, int B, int H, int W, float* x_hat, float* y_lik,
                 float* z_lik, float vbr_scale) {
  return guard([&] {
    MLIC_CHECK(m && x && B > 0, "bad arguments");
    const std::vector<float> sc(B, vbr_scale);
    impl(m).forward(x, B, H, W, x_hat, y_lik, z_lik, sc.data(), (hipStream_t)stream);
  });
}

int mlic_forward_v(mlic_model* m, void* stream, const float* x, int B, int H, int W, float* x_hat, float* y_lik,
                   float* z_lik, const float* vbr_scales) {
  return guard([&] {
    MLIC_CHECK(m && x && B > 0, "bad arguments");
    impl(m).forward(x, B, H, W, x_hat, y_lik, z_lik, vbr_scales, (hipStream_t)stream);
  });
}

int mlic_set_entropy_tables(mlic_model* m, const int32_t* gc_cdf, const int32_t* gc_len, const int32_t* gc_off,
                            int gc_n, int gc_stride, const int32_t* eb_cdf, const int32_t* eb_len,
                            const int32_t* eb_off, int eb_n, int eb_stride) {
  return guard([&] {
    MLIC_CHECK(m, "null model");
    impl(m).set_tables(make_tables(gc_cdf, gc_len, gc_off, gc_n, gc_stride),
                        make_tables(eb_cdf, eb_len, eb_off, eb_n, eb_stride));
  });
}

int mlic_compress(mlic_model* m, void* stream, const float* x, int B, int H, int W, float vbr_scale) {
  return guard([&] {
    MLIC_CHECK(m && x && B > 0, "bad arguments");
    const std::vector<float> sc(B, vbr_scale);
    impl(m).compress(x, B, H, W, sc.data(), (hipStream_t)stream);
  });
}

int mlic_compress_v(mlic_model* m, void* stream, const float* x, int B, int H, int W, const float* vbr_scales) {
  return guard([&] {
    MLIC_CHECK(m && x && B > 0, "bad arguments");
    impl(m).compress(x, B, H, W, vbr_scales, (hipStream_t)stream);
  });
}

int mlic_encoded_size(mlic_model* m, int b, size_t* y_len, size_t* z_len) {
  return guard([&] {
    const EncodedImage& e = impl(m).encoded(b);
    *y_len = e.y.size();
    *z_len = e.z.size();
  });
}

int mlic_encoded_copy(mlic_model* m, int b, uint8_t* y, uint8_t* z) {
  return guard([&] {
    const EncodedImage& e = impl(m).encoded(b);
    std::memcpy(y, e.y.data(), e.y.size());
    std::memcpy(z, e.z.data(), e.z.size());
  });
}

int mlic_encoded_streams(mlic_model* m, int b, int64_t* n_y, int64_t* n_z, int32_t* y_sym, int32_t* y_idx,
                         int32_t* z_sym) {
  return guard([&] {
    const EncodedImage& e = impl(m).encoded(b);
    *n_y = e.y_in.size();
    *n_z = (int64_t)e.z_sym.size();
    e.y_in.gather(y_sym, y_idx);
    if (z_sym) std::memcpy(z_sym, e.z_sym.data(), e.z_sym.size() * 4);
  });
}

int mlic_encoded_bits(mlic_model* m, int b, double* y_bits, double* z_bits) {
  return guard([&] {
    const EncodedImage& e = impl(m).encoded(b);
    if (y_bits) *y_bits = e.y_bits;
    if (z_bits) *z_bits = e.z_bits;
  });
}


int mlic_decompress_v(mlic_model* m, void* stream, const uint8_t* const* y, const size_t* y_len,
                      const uint8_t* const* z, const size_t* z_len, int B, int hz, int wz, float* x_hat,
                      const float* vbr_scales) {
  return guard([&] {
    MLIC_CHECK(m && y && z && x_hat && B > 0 && hz > 0 && wz > 0, "bad arguments");
    impl(m).decompress(y, y_len, z, z_len, B, hz, wz, x_hat, vbr_scales, (hipStream_t)stream);
  });
}

int mlic_batch_stream(mlic_model* m, int first, int count, uint8_t* out, size_t cap, size_t* len) {
  return guard([&] {
    MLIC_CHECK(m && len, "bad arguments");
    const std::string s = impl(m).batch_stream(first, count);
    *len = s.size();
    if (out) {
      MLIC_CHECK(cap >= s.size(), "batch_stream: buffer too small");
      std::memcpy(out, s.data(), s.size());
    }
  });
}

int mlic_decompress_batch_stream(mlic_model* m, void* stream, const uint8_t* y, size_t y_len, const uint8_t* const* z,
                                 const size_t* z_len, int B, int hz, int wz, float* x_hat, const float* vbr_scales) {
  return guard([&] {
    MLIC_CHECK(m && y && z && x_hat && B > 0 && hz > 0 && wz > 0, "bad arguments");
    const uint8_t* ys[1] = {y};
    const size_t yl[1] = {y_len};
    impl(m).decompress(ys, yl, z, z_len, B, hz, wz, x_hat, vbr_scales, (hipStream_t)stream, true);
  });
}

int mlic_decompress(mlic_model* m, void* stream, const uint8_t* const* y, const size_t* y_len,
                    const uint8_t* const* z, const size_t* z_len, int B, int hz, int wz, float* x_hat,
                    float vbr_scale) {
  const std::vector<float> sc(B > 0 ? B : 0, vbr_scale);
  return mlic_decompress_v(m, stream, y, y_len, z, z_len, B, hz, wz, x_hat, sc.data());
}

int mlic_run_module(mlic_model* m, void* stream, const char* which, int idx, const float* in0, const float* in1,
                    int B, int Cin, int H, int W, float* out) {
  return guard([&] { impl(m).run_module(which, idx, in0, in1, B, Cin, H, W, out, (hipStream_t)stream); });
}

int mlic_workspace_bytes(mlic_model* m, size_t* arena, size_t* weights) {
  return guard([&] {
    *arena = impl(m).arena_bytes();
    *weights = impl(m).weight_bytes();
  });
}

int mlic_set_precision(mlic_model* m, int precision) {
  return guard([&] {
    MLIC_CHECK(precision >= PREC_F32 && precision <= PREC_F16X3_V2, "precision must be 0 (f32), 1 or 2 (f16x3)");
    impl(m).set_precision(precision);
  });
}

int mlic_ab_families(int* built) {
  return guard([&] {
    MLIC_CHECK(built, "null out");
    *built = ab_families_built() ? 1 : 0;
  });
}

int mlic_set_kernel_option(const char* name, int value) {
  return guard([&] {
    MLIC_CHECK(name, "null option name");
    const std::string n = name;
    if (n == "x4_halo") x4_set_halo(value);
    else if (n == "linatt_fused") linatt_set_fused(value);
    else if (n == "dw_strip") dw_set_strip(value);
    else if (n == "x4_splitk") x4_set_splitk(value);
    else if (n == "dwpw2") dwpw2_set(value);
    else if (n == "pw3") pw3_set(value);
    else if (n == "narrow_limit") set_narrow_limit(value);
    else if (n == "chain_nj") chain_set_nj(value);
    else if (n == "ep_half") chain_set_ep_half(value);
    else throw Error("mlic: unknown kernel option " + n);
  });
}

int mlic_set_poison(mlic_model* m, int on) {
  return guard([&] { impl(m).set_poison(on != 0); });
}

int mlic_range_fallbacks(mlic_model* m, int64_t* forward_full, int64_t* forward_gs, int64_t* decompress_gs,
                         int reset) {
  return guard([&] {
    Model::Fallbacks& f = impl(m).fallbacks();
    if (forward_full) *forward_full = f.forward_full.load();
    if (forward_gs) *forward_gs = f.forward_gs.load();
    if (decompress_gs) *decompress_gs = f.decompress_gs.load();
    if (reset) {
      f.forward_full = 0;
      f.forward_gs = 0;
      f.decompress_gs = 0;
    }
  });
}

int mlic_set_synthesis_precision(mlic_model* m, int mode) {
  return guard([&] {
    MLIC_CHECK(mode == 0 || mode == 1, "synthesis precision must be 0 (fp32-faithful) or 1 (fp16 operands)");
    impl(m).set_synthesis_precision(mode);
  });
}

int mlic_set_lanes(mlic_model* m, int lanes) {
  return guard([&] { impl(m).set_lanes(lanes); });
}

int mlic_set_priority_base(mlic_model* m, int base) {
  return guard([&] {
    MLIC_CHECK(base >= 0, "priority base must be >= 0");
    impl(m).set_priority_base(base);
  });
}

int mlic_set_profiling(mlic_model* m, int on) {
  return guard([&] { impl(m).set_profiling(on != 0); });
}

int mlic_profile_read(mlic_model* m, int cat, int64_t* launches, double* ms, double* flops, double* bytes) {
  return guard([&] {
    MLIC_CHECK(cat >= 0 && cat < PCAT_COUNT, "profile category");
    ProfStat s = impl(m).profile_read(cat);
    *launches = s.launches;
    *ms = s.ms;
    *flops = s.flops;
    *bytes = s.bytes;
  });
}

int mlic_profile_layers(mlic_model* m, char* buf, size_t cap, size_t* written) {
  return guard([&] {
    std::string s = impl(m).profile_layers();
    *written = s.size();
    if (buf && cap) {
      const size_t n = std::min(cap - 1, s.size());
      std::memcpy(buf, s.data(), n);
      buf[n] = 0;
    }
  });
}

// conv micro-benchmark: random operands of one layer shape, `iters` launches timed with events.
// impl: 0 = conv_mfma (fp32), 1 = conv_f16x3.  Returns ms per launch and TFLOP/s (algorithmic).
int mlic_bench_conv(int impl, int B, int Cin, int Cout, int H, int W, int K, int stride, int epi, int iters,
                    double* ms_per, double* tflops) {
  return guard([&] {
    const int pad = K / 2;
    const int Ho = (H + 2 * pad - K) / stride + 1, Wo = (W + 2 * pad - K) / stride + 1;
    const int64_t nx = (int64_t)B * Cin * H * W, ny = (int64_t)B * Cout * Ho * Wo, nw = (int64_t)Cout * Cin * K * K;
    const int cin_pad = (Cin + 31) / 32 * 32;
    const int64_t nh = (int64_t)Cout * K * K * cin_pad;
    float *x, *y, *w, *wp, *bias;
    _Float16 *wh, *wl;
    HIP_OK(hipMalloc(&x, nx * 4));
    HIP_OK(hipMalloc(&y, ny * 4));
    HIP_OK(hipMalloc(&w, nw * 4));
    HIP_OK(hipMalloc(&wp, nw * 4));
    HIP_OK(hipMalloc(&bias, Cout * 4));
    HIP_OK(hipMalloc(&wh, nh * 2));
    HIP_OK(hipMalloc(&wl, nh * 2));
    {
      std::vector<float> hx(std::max(nx, nw));
      uint32_t st = 12345;
      for (auto& v : hx) { st = st * 1664525u + 1013904223u; v = ((st >> 9) * (1.0f / 8388608.0f)) - 0.5f; }
      HIP_OK(hipMemcpy(x, hx.data(), nx * 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(w, hx.data(), nw * 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemset(bias, 0, Cout * 4));
    }
    pack_conv(w, wp, Cout, Cin, K * K, nullptr);
    const int wexp = split_weights(w, wh, wl, Cout, Cin, K * K, cin_pad, true, nullptr);
    ConvParams P{};
    P.nseg = 1;
    P.seg[0] = {x, Cin, (int64_t)Cin * H * W};
    P.Cin = Cin; P.H = H; P.W = W; P.Cout = Cout; P.Ho = Ho; P.Wo = Wo; P.K = K; P.stride = stride; P.pad = pad;
    P.wpk = wp; P.bias = bias; P.out = y; P.B = B;
    P.out_bs = (int64_t)Cout * Ho * Wo;
    P.out_cs = (int64_t)Ho * Wo;
    P.epi = epi;
    MLIC_CHECK(!(epi & (EPI_GDN | EPI_IGDN | EPI_SHUFFLE)) || !(epi & EPI_RES), "bench: unsupported epilogue");
    if (epi & (EPI_GDN | EPI_IGDN)) {  // the conv input doubles as the GDN operand (Cin == Cout)
      MLIC_CHECK(Cin == Cout && stride == 1, "bench: GDN needs Cin == Cout");
      P.aux = x;
      P.aux_bs = (int64_t)Cin * H * W;
    }
    if (epi & EPI_RES) {  // in place, as the LRP head's residual into y_hat
      P.res = y;
      P.res_bs = P.out_bs;
    }
    _Float16 *wx = nullptr, *wxh = nullptr;
    if (conv_x4_ok(P, cin_pad)) {
      HIP_OK(hipMalloc((void**)&wx, x4_weight_halves(Cout, K * K, cin_pad) * 2));
      x4_pack_weights(wh, wl, Cout, K * K, cin_pad, wx, nullptr);
      if (impl == CONV_X4H) {
        HIP_OK(hipMalloc((void**)&wxh, x4_weight_halves(Cout, K * K, cin_pad, true) * 2));
        x4_pack_weights(wh, wl, Cout, K * K, cin_pad, wxh, nullptr, true);
      }
    }
    ConvWeights cw{wp, wh, wl, cin_pad, wx, wexp};
    cw.wx4h = wxh;
    const int which = impl < 0 ? conv_select(P, cw, 2) : impl;  // < 0: what the model runs (precision 2)
    if (which == CONV_X4H) MLIC_CHECK(conv_x4_ok(P, cin_pad), "x4: unsupported shape");
    if (which == CONV_PW) MLIC_CHECK(pw_resident_ok(P, cin_pad), "pw_resident: unsupported shape");
    if (which == CONV_X4) MLIC_CHECK(conv_x4_ok(P, cin_pad), "x4: unsupported shape");
    void* ws = nullptr;
    const int64_t wsb = conv_ws_bytes(which, P, cw);
    if (wsb > 0) HIP_OK(hipMalloc(&ws, wsb));
    auto launch = [&] { conv_run(which, P, cw, nullptr, ws); };
    launch();
    HIP_OK(hipDeviceSynchronize());
    hipEvent_t a, b;
    HIP_OK(hipEventCreate(&a));
    HIP_OK(hipEventCreate(&b));
    HIP_OK(hipEventRecord(a, nullptr));
    for (int i = 0; i < iters; ++i) launch();
    HIP_OK(hipEventRecord(b, nullptr));
    HIP_OK(hipEventSynchronize(b));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, a, b));
    *ms_per = ms / iters;
    *tflops = 2.0 * (double)B * Cout * Ho * Wo * Cin * K * K / (*ms_per * 1e-3) / 1e12;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (void* p : {(void*)x, (void*)y, (void*)w, (void*)wp, (void*)bias, (void*)wh, (void*)wl, (void*)wx, (void*)wxh, ws})
      if (p) (void)hipFree(p);
  });
}

int mlic_host_stats(mlic_model* m, double* enc_ms, double* dec_ms, double* wait_ms, int reset) {
  return guard([&] {
    HostStats& h = impl(m).host_stats();
    *enc_ms = h.enc_ns.load() * 1e-6;
    *dec_ms = h.dec_ns.load() * 1e-6;
    *wait_ms = h.wait_ns.load() * 1e-6;
    if (reset) {
      h.enc_ns = 0;
      h.dec_ns = 0;
      h.wait_ns = 0;
    }
  });
}

int mlic_profile_categories(int* n) {
  return guard([&] { *n = PCAT_COUNT; });
}

int mlic_profile_category_name(int cat, char* buf, size_t cap) {
  return guard([&] {
    MLIC_CHECK(cat >= 0 && cat < PCAT_COUNT, "profile category");
    const std::string nm = prof_cat_name(cat);
    MLIC_CHECK(cap > nm.size(), "buffer too small");
    std::memcpy(buf, nm.c_str(), nm.size() + 1);
  });
}

int mlic_conv_choice(int B, int Cin, int Cout, int H, int W, int K, int stride, int epi, int* impl) {
  return guard([&] {
    MLIC_CHECK(impl && B > 0 && Cin > 0 && Cout > 0 && H > 0 && W > 0 && (K == 1 || K == 3 || K == 5) && stride > 0,
               "conv_choice: bad arguments");
    const int pad = K / 2;
    ConvParams P{};
    P.nseg = 1;
    P.seg[0] = {nullptr, Cin, (int64_t)Cin * H * W};
    P.Cin = Cin; P.H = H; P.W = W; P.Cout = Cout; P.K = K; P.stride = stride; P.pad = pad;
    P.Ho = (H + 2 * pad - K) / stride + 1;
    P.Wo = (W + 2 * pad - K) / stride + 1;
    P.B = B;
    P.epi = epi;
    const int cin_pad = (Cin + 31) / 32 * 32;
    // weight pointers only signal presence, by the model's own allocation rule (model.cpp: split
    // fp16 copies for Cin >= 16, x4 images of those for K in {1, 3, 5} and Cout >= 64)
    static const _Float16 tag = 0;
    const bool split = Cin >= 16;
    const bool x4 = split && Cout >= 64;
    const ConvWeights cw{nullptr, split ? &tag : nullptr, split ? &tag : nullptr, cin_pad, x4 ? &tag : nullptr, 0};
    *impl = conv_select(P, cw, 2);
  });
}

int mlic_conv_run(void* stream, int impl, const float* x, const float* w, const float* bias, float* y, int B, int Cin,
                  int Cout, int H, int W, int K, int stride, int epi, const float* aux, const float* res) {
  return guard([&] {
    hipStream_t st = (hipStream_t)stream;
    const int pad = K / 2;
    const int Ho = (H + 2 * pad - K) / stride + 1, Wo = (W + 2 * pad - K) / stride + 1;
    const int cin_pad = (Cin + 31) / 32 * 32;
    const int64_t nw = (int64_t)Cout * Cin * K * K, nh = (int64_t)Cout * K * K * cin_pad;
    float* wp = nullptr;
    _Float16 *wh = nullptr, *wl = nullptr;
    HIP_OK(hipMallocAsync((void**)&wp, nw * 4, st));
    HIP_OK(hipMallocAsync((void**)&wh, nh * 2, st));
    HIP_OK(hipMallocAsync((void**)&wl, nh * 2, st));
    pack_conv(w, wp, Cout, Cin, K * K, st);
    const int wexp = split_weights(w, wh, wl, Cout, Cin, K * K, cin_pad, true, st);
    ConvParams P{};
    P.nseg = 1;
    P.seg[0] = {x, Cin, (int64_t)Cin * H * W};
    P.Cin = Cin; P.H = H; P.W = W; P.Cout = Cout; P.Ho = Ho; P.Wo = Wo; P.K = K; P.stride = stride; P.pad = pad;
    P.wpk = wp; P.bias = bias; P.out = y; P.B = B; P.epi = epi;
    const bool shuffle = (epi & EPI_SHUFFLE) != 0;
    MLIC_CHECK(!shuffle || Cout % 4 == 0, "shuffle needs Cout % 4 == 0");
    P.out_cs = shuffle ? (int64_t)4 * Ho * Wo : (int64_t)Ho * Wo;
    P.out_bs = (int64_t)Cout * Ho * Wo;
    MLIC_CHECK(!(epi & (EPI_GDN | EPI_IGDN)) || aux, "GDN epilogue needs aux");
    MLIC_CHECK(!(epi & EPI_RES) || res, "residual epilogue needs res");
    P.aux = aux; P.aux_bs = (int64_t)Cout * Ho * Wo;
    P.res = res; P.res_bs = P.out_bs;
    _Float16 *wx = nullptr, *wxh = nullptr;
    if (conv_x4_ok(P, cin_pad)) {
      HIP_OK(hipMallocAsync((void**)&wx, x4_weight_halves(Cout, K * K, cin_pad) * 2, st));
      x4_pack_weights(wh, wl, Cout, K * K, cin_pad, wx, st);
      if (impl == CONV_X4H) {
        HIP_OK(hipMallocAsync((void**)&wxh, x4_weight_halves(Cout, K * K, cin_pad, true) * 2, st));
        x4_pack_weights(wh, wl, Cout, K * K, cin_pad, wxh, st, true);
      }
    }
    ConvWeights cw{wp, wh, wl, cin_pad, wx, wexp};
    cw.wx4h = wxh;
    const int which = impl < 0 ? conv_select(P, cw, 2) : impl;
    if (which == CONV_X4H) MLIC_CHECK(conv_x4_ok(P, cin_pad), "x4: unsupported shape");
    if (which == CONV_PW) MLIC_CHECK(pw_resident_ok(P, cin_pad), "pw_resident: unsupported shape");
    if (which == CONV_NARROW) MLIC_CHECK(conv_narrow_ok(P), "narrow: unsupported shape");
    if (which == CONV_SMALLCIN) MLIC_CHECK(conv_smallcin_ok(P), "smallcin: unsupported shape");
    if (which == CONV_HALO) MLIC_CHECK(conv_halo_ok(P, cin_pad), "halo: unsupported shape");
    if (which == CONV_X4) MLIC_CHECK(conv_x4_ok(P, cin_pad), "x4: unsupported shape");
    void* ws = nullptr;
    const int64_t wsb = conv_ws_bytes(which, P, cw);
    if (wsb > 0) HIP_OK(hipMallocAsync(&ws, wsb, st));
    conv_run(which, P, cw, st, ws);
    if (ws) HIP_OK(hipFreeAsync(ws, st));
    if (wx) HIP_OK(hipFreeAsync(wx, st));
    if (wxh) HIP_OK(hipFreeAsync(wxh, st));
    HIP_OK(hipFreeAsync(wp, st));
    HIP_OK(hipFreeAsync(wh, st));
    HIP_OK(hipFreeAsync(wl, st));
    HIP_OK(hipStreamSynchronize(st));
  });
}

int mlic_dw_run(void* stream, const float* x, const float* w, const float* bias, float* y, int B, int C, int H, int W,
                int stride, int gelu) {
  return guard([&] {
    DwParams P{};
    P.nseg = 1;
    P.seg[0] = {x, C, (int64_t)C * H * W};
    P.C = C; P.H = H; P.W = W; P.stride = stride;
    P.Ho = (H - 1) / stride + 1;
    P.Wo = (W - 1) / stride + 1;
    P.w = w; P.bias = bias; P.out = y; P.out_bs = (int64_t)C * P.Ho * P.Wo; P.gelu = gelu; P.B = B;
    dw3x3(P, (hipStream_t)stream);
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  });
}

int mlic_dwpw_run(void* stream, const float* x, const float* dww, const float* dwb, const float* w, const float* bias,
                  float* y, int B, int C, int Cout, int H, int W, int epi, const float* res) {
  return guard([&] {
    hipStream_t st = (hipStream_t)stream;
    const int cin_pad = (C + 31) / 32 * 32;
    const int64_t nh = (int64_t)Cout * cin_pad;
    _Float16 *wh = nullptr, *wl = nullptr;
    HIP_OK(hipMallocAsync((void**)&wh, nh * 2, st));
    HIP_OK(hipMallocAsync((void**)&wl, nh * 2, st));
    const int wexp = split_weights(w, wh, wl, Cout, C, 1, cin_pad, true, st);
    ConvParams P{};
    P.nseg = 1;
    P.seg[0] = {x, C, (int64_t)C * H * W};
    P.Cin = C; P.H = H; P.W = W; P.Cout = Cout; P.Ho = H; P.Wo = W; P.K = 1; P.stride = 1; P.pad = 0;
    P.wexp = wexp; P.bias = bias; P.out = y; P.B = B; P.epi = epi;
    P.out_cs = (int64_t)H * W;
    P.out_bs = (int64_t)Cout * H * W;
    MLIC_CHECK(!(epi & EPI_RES) || res, "residual epilogue needs res");
    P.res = res; P.res_bs = P.out_bs;
    MLIC_CHECK(dwpw_ok(P, cin_pad), "dwpw: unsupported shape");
    dwpw_forward(P, wh, wl, cin_pad, dww, dwb, st);
    HIP_OK(hipFreeAsync(wh, st));
    HIP_OK(hipFreeAsync(wl, st));
    HIP_OK(hipStreamSynchronize(st));
  });
}

int mlic_local_attn_run(void* stream, int impl, const float* qkv, const float* rel_table, const int32_t* rel_index,
                        float* out, int C, int H, int W, int B, float scale) {
  return guard([&] {
    LocalAttnParams A{};
    A.qkv = qkv;
    A.qkv_bs = (int64_t)3 * C * H * W;
    A.out = out;
    A.out_bs = (int64_t)25 * C * H * W;
    A.rel_table = rel_table;
    A.rel_index = rel_index;
    A.scale = scale;
    A.C = C; A.H = H; A.W = W; A.B = B;
    if (impl == 0) local_attn_valu(A, (hipStream_t)stream);
    else local_attn_mfma(A, (hipStream_t)stream);
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  });
}

int mlic_local_attn_packed_run(void* stream, const float* qkv, const float* rel_table, const int32_t* rel_index,
                               uint16_t* out, int H, int W, int B, float scale) {
  return guard([&] {
    LocalAttnParams A{};
    A.qkv = qkv;
    A.qkv_bs = (int64_t)3 * 32 * H * W;
    A.rel_table = rel_table;
    A.rel_index = rel_index;
    A.scale = scale;
    A.C = 32; A.H = H; A.W = W; A.B = B;
    local_attn_packed(A, reinterpret_cast<_Float16*>(out), (H * W + 31) / 32 * 32, (hipStream_t)stream);
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  });
}

int mlic_local_attn_packed_half_run(void* stream, const float* qkv, const float* rel_table, const int32_t* rel_index,
                                    uint16_t* out, int H, int W, int B, float scale, int ckbd) {
  return guard([&] {
    MLIC_CHECK(ckbd == 1 || ckbd == 2, "ckbd: 1 (anchors) or 2 (non-anchors)");
    LocalAttnParams A{};
    A.qkv = qkv;
    A.qkv_bs = (int64_t)3 * 32 * H * W;
    A.rel_table = rel_table;
    A.rel_index = rel_index;
    A.scale = scale;
    A.C = 32; A.H = H; A.W = W; A.B = B;
    A.ckbd = ckbd;
    local_attn_packed(A, reinterpret_cast<_Float16*>(out), (H * W / 2 + 31) / 32 * 32, (hipStream_t)stream);
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  });
}

int mlic_local_attn_mask(void* stream, float* out, int H, int W) {
  return guard([&] { local_mask(out, H, W, (hipStream_t)stream); });
}

int mlic_image_sq_err_u8(void* stream, const float* a, const float* b, int B, int64_t n_per, double* out) {
  return guard([&] { sq_err_u8(a, n_per, b, n_per, out, n_per, B, (hipStream_t)stream); });
}

int mlic_neglog2_sum(void* stream, const float* lik, int B, int64_t n_per, double* out) {
  return guard([&] {
    double* part = nullptr;
    HIP_OK(hipMalloc(&part, sizeof(double) * neglog2_partial_doubles(B)));
    try {
      neglog2_sum(lik, n_per, B, out, part, (hipStream_t)stream);
      HIP_OK(hipStreamSynchronize((hipStream_t)stream));
    } catch (...) {
      (void)hipFree(part);
      throw;
    }
    HIP_OK(hipFree(part));
  });
}

int mlic_gaussian_likelihood(void* stream, const float* y, const float* scales, const float* means, int64_t n,
                             float vbr_scale, float* lik) {
  return guard([&] {
    MLIC_CHECK(n >= 0 && (n == 0 || (y && scales && means && lik)), "gaussian_likelihood arguments");
    gauss_likelihood(y, scales, means, n, vbr_scale, lik, (hipStream_t)stream);
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  });
}

int mlic_scale_indexes(void* stream, const float* scales, int64_t n, const float* table, int ntable, int32_t* out) {
  return guard([&] {
    MLIC_CHECK(ntable >= 2 && ntable <= 1024, "scale table size");
    MLIC_CHECK(n >= 0 && (n == 0 || (scales && table && out)), "scale_indexes arguments");
    scale_indexes(scales, n, table, ntable, out, (hipStream_t)stream);
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  });
}

int mlic_pmf_to_quantized_cdf(const float* pmf, int n, int precision, int32_t* cdf_out) {
  return guard([&] {
    auto c = pmf_to_quantized_cdf(pmf, n, precision);
    for (size_t i = 0; i < c.size(); ++i) cdf_out[i] = (int32_t)c[i];
  });
}

int mlic_rans_encode(const int32_t* symbols, const int32_t* indexes, int64_t n, const int32_t* cdf,
                     const int32_t* cdf_len, const int32_t* offset, int n_tables, int stride, uint8_t* out,
                     size_t cap, size_t* written) {
  return guard([&] {
    CdfTables t = make_tables(cdf, cdf_len, offset, n_tables, stride);
    std::string s = rans_encode(symbols, indexes, n, t);
    *written = s.size();
    MLIC_CHECK(s.size() <= cap, "output buffer too small");
    std::memcpy(out, s.data(), s.size());
  });
}

int mlic_rans_decode(const uint8_t* data, size_t nbytes, const int32_t* indexes, int64_t n, const int32_t* cdf,
                     const int32_t* cdf_len, const int32_t* offset, int n_tables, int stride, int32_t* out) {
  return guard([&] {
    CdfTables t = make_tables(cdf, cdf_len, offset, n_tables, stride);
    RansDecoderState d;
    d.set_stream(data, nbytes);
    d.decode(indexes, n, t, out);
  });
}

int mlic_rans_decode_narrow(const uint8_t* data, size_t nbytes, const uint8_t* indexes, int64_t n, int nparts,
                            const int32_t* cdf, const int32_t* cdf_len, const int32_t* offset, int n_tables,
                            int stride, int32_t* out, int* widened) {
  return guard([&] {
    MLIC_CHECK(nparts >= 1 && n % nparts == 0 && widened, "rans_decode_narrow: n / nparts");
    CdfTables t = make_tables(cdf, cdf_len, offset, n_tables, stride);
    RansDecoderState d;
    d.set_stream(data, nbytes);
    const int64_t np = n / nparts;
    std::vector<int16_t> s16(np);
    *widened = 0;
    for (int k = 0; k < nparts; ++k) {
      if (rans_decode_piece(d, indexes + k * np, np, t, s16.data(), out + k * np))
        for (int64_t i = 0; i < np; ++i) out[k * np + i] = s16[i];
      else
        ++*widened;
    }
  });
}

}  // extern "C"
