// MLIC++ model executor: the reference's module graph (models/mlicpp.py, mlicpp_small_decoder.py,
// mlicpp_vbr.py) driven natively over the HIP kernels, on one stream, with a per-handle arena.
#pragma once
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "pool.h"
#include "rans.h"

namespace mlic {

struct Cfg {
  std::string name;
  int N = 0, M = 0, S = 0, C = 0, win = 5;
  bool sd = false, vbr = false;
  int hM() const { return sd ? M / 4 : M; }
  int gN() const { return sd ? N / 4 : N; }
};
Cfg config_for(const std::string& name);

struct ConvW {
  float* w = nullptr;        // packed [K*K][Cin][Cout]            (fp32 MFMA path)
  const float* b = nullptr;  // [Cout] or null
  int Cin = 0, Cout = 0, K = 0;
  _Float16* wh = nullptr;    // split hi/lo [Cout][K*K][cin_pad]  (f16x3 MFMA path)
  _Float16* wl = nullptr;
  int cin_pad = 0;
  _Float16* wx4 = nullptr;   // x4 LDS-image weights [ct][step][BM][64]     (conv_x4 path)
  _Float16* wx4h = nullptr;  // reduced-precision x4 image (64 channels of hi per row; g_s subpel convs)
  int wexp = 0;              // wh/wl hold w * 2^wexp (exact layer prescale, split_weights)
  std::string name;          // state_dict prefix (profiling)
};

// a fused 1x1 chain (chain.hip): EntropyParameters' 4 layers or LocalContext's MLP
struct ChainW {
  _Float16* wimg = nullptr;  // per-layer LDS images, concatenated
  int nl = 0, cin0 = 0;
  int cout[4] = {0, 0, 0, 0};
  const float* bias[4] = {nullptr, nullptr, nullptr, nullptr};
  int wexp[4] = {0, 0, 0, 0};
  std::string name;
};

enum Precision : int { PREC_F32 = 0, PREC_F16X3 = 1, PREC_F16X3_V2 = 2 };
struct DwW {
  const float* w = nullptr;  // [C][9]
  const float* b = nullptr;
  int C = 0;
  std::string name;
};

// arena: stream-ordered bump allocator; a dry run sizes it
class Arena {
 public:
  ~Arena();
  void ensure(size_t bytes);
  float* alloc(int64_t nfloats);
  size_t mark() const { return top_; }
  void release(size_t m) { top_ = m; }
  void begin(bool dry) { dry_ = dry; top_ = 0; peak_ = 0; }
  size_t peak() const { return peak_; }
  size_t capacity() const { return cap_; }
  // test switch ($MLIC_POISON / mlic_set_poison): every block handed out by alloc() is filled with
  // 0xFF bytes (a NaN in every fp32 / fp16 lane) on `st` first, so a kernel that reads arena memory
  // its producer never wrote poisons its output instead of silently reading a previous call's data
  void poison_on(hipStream_t st) { poison_st_ = st; poison_ = true; }
  void poison_off() { poison_ = false; }

 private:
  char* base_ = nullptr;
  size_t cap_ = 0, top_ = 0, peak_ = 0;
  bool dry_ = false;
  bool poison_ = false;
  hipStream_t poison_st_ = nullptr;
};

// live per-kernel-family timing with HIP events on the executor's stream (bench.py roofline);
// categories: ProfCat in kernels.h
struct ProfStat {
  int64_t launches = 0;
  double ms = 0, flops = 0, bytes = 0;
};

// An image's y coder inputs where compress left them: the lane's pinned phase-major buffers
// ([phase][B][n_per]), valid until the model's next compress().  Symbols are int16 (sym16) unless one
// of the call's symbols did not fit (then sym, int32); indexes are uint8.
struct CoderView {
  const int32_t* sym = nullptr;
  const int16_t* sym16 = nullptr;
  const uint8_t* idx = nullptr;
  int64_t n_per = 0, stride = 0;  // symbols per phase of one image; distance between phases
  int nph = 0;
  int64_t size() const { return n_per * nph; }
  void gather(int32_t* s, int32_t* i) const {  // coder order: phases in order, widened to int32
    for (int k = 0; k < nph; ++k) {
      for (int64_t j = 0; j < n_per; ++j) {
        if (s) s[k * n_per + j] = sym16 ? (int32_t)sym16[k * stride + j] : sym[k * stride + j];
        if (i) i[k * n_per + j] = (int32_t)idx[k * stride + j];
      }
    }
  }
  // rANS-code phase k into e (RansEncoder::put_reverse in the stored widths)
  template <class E, class T>
  void put_phase(E& e, int k, const T& tables) const {
    if (sym16) e.put_reverse(sym16 + k * stride, idx + k * stride, n_per, tables);
    else e.put_reverse(sym + k * stride, idx + k * stride, n_per, tables);
  }
};

// device-side coder buffers of one call: encoder [phase][B][n_per] (sym int32 always, sym16 / idx8 the
// narrow copies that leave for the host, ovf the int16 overflow flag); decoder [B][n_per] of one phase
struct CoderBufs {
  int32_t* sym = nullptr;
  int16_t* sym16 = nullptr;
  uint8_t* idx8 = nullptr;
  int* ovf = nullptr;
};

struct EncodedImage {
  std::string y;  // one rANS stream for all slices/phases
  std::string z;  // z stream (EntropyBottleneck)
  CoderView y_in;              // the y coder inputs (tests / tooling / batch_stream)
  std::vector<int32_t> z_sym;  // the z coder inputs
  double y_bits = 0, z_bits = 0;  // sum of -log2 of the y / z likelihoods (rd_loss.py:42-45 numerator)
};

class PhaseDecoder;

// host-side time accounting (summed over threads): entropy coding and waits on the GPU
struct HostStats {
  std::atomic<int64_t> enc_ns{0}, dec_ns{0}, wait_ns{0};
  struct Scope {
    std::atomic<int64_t>& acc;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~Scope() {
      acc += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
  };
};

// Per-call execution state.  A Model owns several lanes so that a batch can be split over host
// threads, each driving its own HIP stream: one lane's host entropy coding overlaps another
// lane's kernels (weights and entropy tables are shared, read-only).
struct Lane {
  Arena arena;
  hipStream_t st = nullptr;
  bool own_stream = false;
  int B = 0;
  bool dry = false;
  std::vector<float> vbr_host;  // [2][B]: per-image gain, then 1 / gain (uploaded by slice_loop)
  bool vbr_on = false;
  std::vector<EncodedImage> enc;
  int32_t* h_sym = nullptr;    // decoder: z symbols; a phase's symbols when one does not fit int16
  int16_t* h_sym16 = nullptr;  // decoder: a phase's symbols (H2D)
  uint8_t* h_idx8 = nullptr;   // decoder: a phase's scale indexes (D2H)
  size_t h_cap = 0;
  // compress: every phase's symbols / indexes leave for these pinned buffers on the copy stream as
  // soon as the phase is quantised, so only the last phase's copy is left when the network ends
  hipStream_t cst = nullptr;
  hipEvent_t cev = nullptr;
  int32_t* hc_sym = nullptr;    // z symbols; the y symbols when one of them did not fit int16
  int16_t* hc_sym16 = nullptr;  // y symbols
  uint8_t* hc_idx8 = nullptr;   // y scale indexes
  size_t hc_cap = 0;
  bool phase_d2h = false;
  // profiling
  struct ProfRec {
    hipEvent_t a, b;
    int cat;
    double flops, bytes;
    std::string tag;
  };
  bool prof = false;
  int* rflag = nullptr;  // this lane's device fp16 range flag (common.h range_check)
  int prec_force = -1;   // >= 0: arithmetic override for this lane's current call (range-guard fallbacks)
  std::vector<ProfRec> recs;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  ~Lane();
};

class Model {
 public:
  Model(const std::string& name, int n, const char* const* names, const float* const* ptrs, const int64_t* shapes,
        const int* ndims, hipStream_t st);
  ~Model();
  const Cfg& cfg() const { return cfg_; }
  HostStats& host_stats() { return hstats_; }
  HostPool& host_pool();  // shared entropy-coding workers ($MLIC_HOST_THREADS, <= 16)

  // forward(): x [B,3,H,W] -> x_hat, y_lik [B,M,H/16,W/16], z_lik [B,N,H/64,W/64] (any may be null)
  // vbr_scales: per-image Gain (host array of B; null = 1 for all); only *_VBR models use it
  void forward(const float* x, int B, int H, int W, float* x_hat, float* y_lik, float* z_lik, const float* vbr_scales,
               hipStream_t st);
  // compress(): network + rANS; results readable with encoded(b)
  void compress(const float* x, int B, int H, int W, const float* vbr_scales, hipStream_t st);
  const EncodedImage& encoded(int b) const { return enc_all_.at(b); }
  // decompress(): y/z byte streams per image -> x_hat [B,3,4*16*hz,4*16*wz]
  // batch_stream: y[0] is ONE stream holding the whole batch in the reference's order (mlicpp.py:215,
  // 279-281: phase-major, image-minor); decoded on one lane (the stream is sequential)
  void decompress(const uint8_t* const* y, const size_t* ylen, const uint8_t* const* z, const size_t* zlen, int B,
                  int hz, int wz, float* x_hat, const float* vbr_scales, hipStream_t st, bool batch_stream = false);
  // the last compress()'s images [first, first + count) coded into ONE y stream in the reference's
  // batched order (mlicpp.py:215, 279-281): byte-identical to what the reference's compress() emits for
  // that batch when it codes the same symbols
  std::string batch_stream(int first, int count) const;
  void set_tables(const CdfTables& gc, const CdfTables& eb) {
    gc_ = gc;
    eb_ = eb;
  }
  size_t arena_bytes() const;
  void set_profiling(bool on);
  void set_lanes(int n);
  void set_precision(int p) { precision_ = p; }
  int precision() const { return precision_; }
  // g_s's dense subpel convs: 0 = fp32-faithful (the model precision), 1 = fp16 operands with fp32
  // accumulation (decoder output only: bitstreams and likelihoods do not change)
  void set_synthesis_precision(int p) { gs_fp16_ = p == 1; }
  int synthesis_precision() const { return gs_fp16_ ? 1 : 0; }
  int lanes() const { return nlanes_; }
  // stream-priority offset of this model's lanes (lane i: greatest + base + i, clamped): request streams
  // served by separate models get staggered priorities too (applies to lanes created afterwards)
  void set_priority_base(int b) { prio_base_ = b; }
  // test switch: NaN-fill every arena block on allocation (Arena::poison_on); also $MLIC_POISON=1
  void set_poison(bool on) { poison_ = on; }
  // fp16 range-guard fallbacks taken since the last reset (they change the arithmetic of a call, so the
  // round-trip tests assert they are 0): forward re-run whole in exact fp32 (the entropy model left
  // fp16's range), forward's g_s alone, decompress's g_s alone
  struct Fallbacks {
    std::atomic<int64_t> forward_full{0}, forward_gs{0}, decompress_gs{0};
  };
  Fallbacks& fallbacks() { return fb_; }
  ProfStat profile_read(int cat);  // synchronises the recorded events; clears that category
  std::string profile_layers();     // per-tag table of the recorded events (does not clear)
  size_t weight_bytes() const { return wbytes_; }
  // module-level entry points for tests
  void run_module(const std::string& which, int idx, const float* in0, const float* in1, int B, int Cin, int H, int W,
                  float* out, hipStream_t st);

 private:
  enum class Mode { Forward, Encode, Decode };
  Cfg cfg_;
  std::map<std::string, ConvW> convs_;
  std::map<std::string, ChainW> chains_;  // keyed by the module prefix (".fusion" / ".mlp")
  // EntropyParameters with the hyper columns of layer 0 hoisted out of the slice loop: one GEMM
  // W_hyp (all 2 S EPs stacked, 2 S x 320 rows) . hyper per image before the loop; the chains_ctx_
  // then run layer 0 over the context channels only and start from the hoisted rows (aux)
  std::map<std::string, ChainW> chains_ctx_;
  ConvW hoist_;          // stacked [2 S x C1][2 hM] (Cout = 0: no hoisting)
  int hoist_rows_ = 0;   // C1 (320)
  bool hoist_on() const;
  void add_hoist(const std::map<std::string, std::pair<const float*, int>>& ep0, hipStream_t st);
  ConvW make_conv(const float* w_dev, int Cout, int Cin, int K, const std::string& name, hipStream_t st);
  void add_chains(hipStream_t st);
  // the lane's fp16 range flag: read and clear (synchronises the lane stream), clear (stream-ordered)
  bool range_hit(Lane& l);
  void range_clear(Lane& l);
  int prec() const { return L().prec_force >= 0 ? L().prec_force : precision_; }
  void run_chain(const ChainW& c, const std::vector<View>& ins, const View& out, const View* res,
                 const View* aux = nullptr, int H = 0, int W = 0, int ckbd = 0, bool sq_in = false);
  bool chain_on() const;
  bool dwpw_on() const;
  std::map<std::string, DwW> dws_;
  std::map<std::string, const float*> raw_;
  std::vector<void*> owned_;
  size_t wbytes_ = 0;
  float* scale_table_ = nullptr;
  int* rel_index_ = nullptr;
  CdfTables gc_, eb_;
  std::vector<EncodedImage> enc_all_;
  std::vector<std::unique_ptr<Lane>> lanes_;
  int nlanes_ = 4;
  int prio_base_ = 0;
  int precision_ = PREC_F16X3_V2;
  bool gs_fp16_ = false;
  HostStats hstats_;
  bool prof_ = false;
  bool poison_ = false;
  Fallbacks fb_;
  // re-run g_s alone in exact fp32 MFMA from a copy of y_hat (the re-plan may move the arena)
  void gs_fp32_rerun(Lane& l, const View& yhat, const View& out, int B);
  static thread_local Lane* tl_lane_;
  Lane& L() const { return *tl_lane_; }
  Lane& lane(int i);
  hipEvent_t next_event();
  template <class F>
  void timed(int cat, double flops, double bytes, F&& launch, const std::string& tag = std::string());
  // run fn(lane, first_image, count) over the batch split across lanes (host threads)
  template <class F>
  void over_lanes(int B, hipStream_t caller, F&& fn, int max_lanes = 16);
  void compress_lane(const float* x, int B, int H, int W);
  void decompress_lane(const uint8_t* const* y, const size_t* ylen, const uint8_t* const* z, const size_t* zlen,
                       int B, int hz, int wz, float* x_hat, bool batch_stream);

  // -- weights
  const ConvW& cw(const std::string& k) const;
  const DwW& dww(const std::string& k) const;
  const float* rw(const std::string& k) const;
  bool has(const std::string& k) const { return convs_.count(k) || dws_.count(k) || raw_.count(k); }

  // -- building blocks (outputs allocated in the arena unless given)
  View alloc(int C, int H, int W);
  void conv(const std::vector<View>& ins, const ConvW& w, int stride, int pad, const View& out, int epi,
            const View* aux = nullptr, const View* res = nullptr);
  ConvParams conv_params(const std::vector<View>& ins, const ConvW& w, int stride, int pad, const View& out, int epi,
                         const View* aux, const View* res);
  void run_conv(const ConvParams& P, const ConvW& w, const _Float16* packed, bool hi = false, bool split = false);
  void linatt_reproject(const View& k, const View& v, const View& q, int heads, int hd, int kmask, int qmask,
                        const ConvW& rp, const View& a, const std::string& tag);
  void add_fusion_x4(const std::string& base, const float* w_dev, int Cout, hipStream_t st);
  void add_taps(const std::string& base, const float* w_dev, int Cin, hipStream_t st);
  bool taps_on() const;
  void conv_pair(const std::vector<View>& ins, const ConvW& w1, const View& out1, int epi1, const ConvW& w2,
                 const View& out2, int epi2);
  void dw(const std::vector<View>& ins, const DwW& w, int stride, const View& out, bool gelu);
  View conv3x3(const std::vector<View>& ins, const std::string& p, int stride, bool dwsep, int epi,
               const View* res = nullptr, const View* out = nullptr);
  View conv1x1(const View& in, const std::string& p, int stride, int epi, const View* res = nullptr);
  void gdn(const View& x, const std::string& p, bool inverse, const View& out, const View* res);
  View rbws(const View& x, const std::string& p, bool dwsep);
  View rb(const View& x, const std::string& p, bool dwsep);
  View rbu(const View& x, const std::string& p);
  View g_a(const View& x);
  View h_a(const View& y);
  View h_s(const View& z_hat);
  void g_s(const View& y_hat, const View& out);
  // half: the output is read at the non-anchor pixels only (the slice loop, when the non-anchor
  // EntropyParameters runs on its half: ep_half_chain) -- attention, fusion, norm and MLP on that half
  View local_context(const View& x, int i, bool half = false);
  // the slice loop's EntropyParameters of (kind, i) will run as a chain over its phase's half of the grid
  bool ep_half_chain(const std::string& kind, int i, int H, int W, bool hoisted) const;
  View channel_context(const View& x, int i);
  View inter_context(const View& x, int i);
  View intra_context(const View& x1, const View& x2, int i);
  // ctx: the context segments of the layer-0 concat (entropy.py), hyper appended last; hoisted: the
  // slice loop's precomputed W_hyp . hyper rows of all EPs (or null); phase_only: the output is read at the
  // kind's own checkerboard pixels only (the slice loop), so the chain may skip the other half
  View entropy_parameters(const std::vector<View>& ctx, const View* hyper, const std::string& kind, int i,
                          const View* hoisted = nullptr, bool phase_only = false);
  void lrp(const std::vector<View>& ins, const std::string& kind, int i, const View& yh_slice, bool anchor);
  View qkv_branch(const View& x, const std::string& p);
  void slice_loop(Mode mode, const View& hyper, const View* y, const View& yhat, float* y_lik, const CoderBufs* cb,
                  class PhaseDecoder* dec);
  void eb(const View& z, const View& z_hat, float* z_lik, int32_t* z_sym);

  template <class F>
  void planned(int B, hipStream_t st, F&& body);
  void ensure_host(size_t n);
  void ensure_chost(size_t n);
  static int phase_d2h_mode();
  void set_vbr(const float* scales, int B);
};

}  // namespace mlic
