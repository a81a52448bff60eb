// MLIC++ executor.  Every method cites the reference code it re-expresses; the arithmetic runs in
// the HIP kernels (conv_mfma.hip, kernels.hip), this file only wires views, weights and phases.
#include "model.h"

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>

namespace mlic {

// g_s's dense 3x3 subpel convs (ResidualBlockUpsample subpel_conv / upsample, res_blk.py:107,111):
// the convs the reduced-precision synthesis mode runs in the single-term fp16 form
static bool gs_subpel(const std::string& name, const ConvW& w) {
  return name.rfind("g_s.", 0) == 0 && w.K == 3 && w.wh != nullptr;
}

// ------------------------------------------------------------------------------------- configs
Cfg config_for(const std::string& name) {  // config/config.py:19-62 (+ MLICPP_L_VBR)
  Cfg c;
  c.name = name;
  if (name == "MLICPP_L" || name == "MLICPP_L_VBR") { c.N = 192; c.M = 320; c.S = 10; }
  else if (name == "MLICPP_S" || name == "MLICPP_S_VBR") { c.N = 96; c.M = 160; c.S = 5; }
  else if (name == "MLICPP_M") { c.N = 160; c.M = 256; c.S = 8; }
  else if (name == "MLICPP_S2") { c.N = 128; c.M = 128; c.S = 2; }
  else if (name == "MLICPP_M_SMALL_DEC" || name == "MLICPP_M_SMALL_DEC_VBR") { c.N = 192; c.M = 320; c.S = 10; c.sd = true; }
  else throw Error("mlic: unknown model name " + name);
  c.vbr = name.size() > 4 && name.substr(name.size() - 4) == "_VBR";
  c.C = c.M / c.S;
  return c;
}

// ------------------------------------------------------------------------------------- arena
Arena::~Arena() {
  if (base_) (void)hipFree(base_);
}

void Arena::ensure(size_t bytes) {
  if (bytes <= cap_) return;
  if (base_) HIP_OK(hipFree(base_));
  base_ = nullptr;
  HIP_OK(hipMalloc(&base_, bytes));
  cap_ = bytes;
}

float* Arena::alloc(int64_t nfloats) {
  const size_t bytes = ((size_t)nfloats * sizeof(float) + 255) & ~(size_t)255;
  const size_t off = top_;
  top_ += bytes;
  peak_ = std::max(peak_, top_);
  if (dry_) return reinterpret_cast<float*>((uintptr_t)0x1000 + off);  // never dereferenced
  MLIC_CHECK(top_ <= cap_, "arena overflow (plan mismatch)");
  if (poison_) HIP_OK(hipMemsetAsync(base_ + off, 0xFF, bytes, poison_st_));
  return reinterpret_cast<float*>(base_ + off);
}

// ------------------------------------------------------------------------------------- weights
static bool ends_with(const std::string& s, const std::string& t) {
  return s.size() >= t.size() && s.compare(s.size() - t.size(), t.size(), t) == 0;
}

Model::Model(const std::string& name, int n, const char* const* names, const float* const* ptrs,
             const int64_t* shapes, const int* ndims, hipStream_t st)
    : cfg_(config_for(name)) {
  // one owned device block for every weight (packed or copied)
  std::vector<int64_t> numel(n);
  size_t total = 0;
  for (int i = 0; i < n; ++i) {
    int64_t e = 1;
    for (int d = 0; d < ndims[i]; ++d) e *= shapes[i * 4 + d];
    numel[i] = e;
    total += ((size_t)e * 4 + 255) & ~(size_t)255;
  }
  for (int i = 0; i < n; ++i) {
    if (ends_with(names[i], ".gamma") && ndims[i] == 2) total += (size_t)(2 * numel[i] + shapes[i * 4]) * 4 + 1024;
    if (ends_with(names[i], ".weight") && (ndims[i] == 4 || ndims[i] == 2)) {
      // split fp16 copy: 2 x Cout x KK x cin_pad halves
      const int64_t cout = shapes[i * 4], per = numel[i] / std::max<int64_t>(1, cout);
      total += (size_t)(cout * (per + 32 * 25)) * 4 + 1024;
    }
  }
  total += 64 * 4 + 625 * 4 + 1024;
  char* block = nullptr;
  HIP_OK(hipMalloc(&block, total));
  owned_.push_back(block);
  wbytes_ = total;
  size_t off = 0;
  auto take = [&](int64_t nf) {
    char* p = block + off;
    off += ((size_t)nf * 4 + 255) & ~(size_t)255;
    return reinterpret_cast<float*>(p);
  };
  std::map<std::string, int> idx;
  for (int i = 0; i < n; ++i) idx[names[i]] = i;
  auto shape = [&](int i, int d) { return (int)shapes[i * 4 + d]; };

  std::map<std::string, std::pair<const float*, int>> ep0;  // EntropyParameters layer-0 weights (hoisting)
  std::vector<CopyDesc> copies;  // plain parameter copies, made by one launch after the loop
  for (int i = 0; i < n; ++i) {
    const std::string k = names[i];
    float* dst = take(numel[i]);
    if (k.rfind("entropy_parameters", 0) == 0 && ends_with(k, ".fusion.0.weight") && ndims[i] == 4)
      ep0[k.substr(0, k.size() - 7)] = {ptrs[i], shape(i, 1)};
    const std::string base = k.substr(0, k.rfind('.'));
    if (ends_with(k, ".weight") && ndims[i] == 4 && shape(i, 1) == 1 && shape(i, 0) > 1) {
      // depthwise [C,1,3,3]
      copies.push_back(CopyDesc{dst, ptrs[i], numel[i]});
      DwW w;
      w.w = dst;
      w.C = shape(i, 0);
      MLIC_CHECK(shape(i, 2) == 3 && shape(i, 3) == 3, "depthwise kernels are 3x3");
      w.name = base;
      dws_[base] = w;
    } else if (ends_with(k, ".weight") && (ndims[i] == 4 || ndims[i] == 2) &&
               k.find("entropy_bottleneck") == std::string::npos && k.find("norm") == std::string::npos) {
      ConvW w;
      w.w = dst;
      w.Cout = shape(i, 0);
      if (ndims[i] == 2) {  // nn.Linear == 1x1 conv
        w.Cin = shape(i, 1);
        w.K = 1;
      } else if (k.find("local_context") != std::string::npos && ends_with(k, ".fusion.weight")) {
        // 5x5 valid conv over the 5x5 window tensor == 1x1 conv over Cin*25 rows (c*25 + cell)
        w.Cin = shape(i, 1) * shape(i, 2) * shape(i, 3);
        w.K = 1;
      } else {
        w.Cin = shape(i, 1);
        w.K = shape(i, 2);
        MLIC_CHECK(shape(i, 2) == shape(i, 3), "square kernels only");
      }
      pack_conv(ptrs[i], dst, w.Cout, w.Cin, w.K * w.K, st);
      if (k.find("local_context") != std::string::npos && ends_with(k, ".fusion.weight") && w.Cin == 800)
        add_fusion_x4(base, ptrs[i], w.Cout, st);
      if (base == "g_s.synthesis_transform.7.0" && w.K == 3 && w.Cout == 12) add_taps(base, ptrs[i], w.Cin, st);
      if (w.Cin >= 16) {  // split-fp16 copy for the f16x3 MFMA path
        w.cin_pad = (w.Cin + 31) / 32 * 32;
        const int64_t nh = (int64_t)w.Cout * w.K * w.K * w.cin_pad;
        w.wh = reinterpret_cast<_Float16*>(take((nh + 1) / 2));
        w.wl = reinterpret_cast<_Float16*>(take((nh + 1) / 2));
        w.wexp = split_weights(ptrs[i], w.wh, w.wl, w.Cout, w.Cin, w.K * w.K, w.cin_pad, true, st);
      }
      w.name = base;
      convs_[base] = w;
    } else {
      copies.push_back(CopyDesc{dst, ptrs[i], numel[i]});
      raw_[k] = dst;
    }
  }
  if (!copies.empty()) {
    // (before any kernel below reads a copied parameter: same stream)
    CopyDesc* dd = nullptr;
    HIP_OK(hipMalloc(&dd, copies.size() * sizeof(CopyDesc)));
    owned_.push_back(dd);
    HIP_OK(hipMemcpyAsync(dd, copies.data(), copies.size() * sizeof(CopyDesc), hipMemcpyHostToDevice, st));
    copy_many(dd, (int)copies.size(), st);
    HIP_OK(hipStreamSynchronize(st));  // the host vector of descriptors dies here
  }
  // biases
  for (auto& kv : convs_) {
    const std::string b = ends_with(kv.first, ".__x4perm") ? kv.first.substr(0, kv.first.size() - 9) : kv.first;
    auto it = raw_.find(b + ".bias");
    if (it != raw_.end()) kv.second.b = it->second;
  }
  for (auto& kv : dws_) {
    auto it = raw_.find(kv.first + ".bias");
    if (it != raw_.end()) kv.second.b = it->second;
  }
  // GDN: eff = max(p, bound)^2 - pedestal; gamma as a 1x1 conv with beta_eff as its bias
  for (int i = 0; i < n; ++i) {
    const std::string k = names[i];
    if (!ends_with(k, ".gamma") || ndims[i] != 2) continue;
    const std::string p = k.substr(0, k.size() - 6);
    const int C = shape(i, 0);
    float* beta_eff = take(C);
    float* gamma_pk = take((int64_t)C * C);
    float* gamma_eff = take((int64_t)C * C);
    MLIC_CHECK(off <= total, "weight block");
    gdn_prep(rw(p + ".beta"), rw(p + ".gamma"), rw(p + ".beta_reparam.lower_bound.bound"),
             rw(p + ".beta_reparam.pedestal"), rw(p + ".gamma_reparam.lower_bound.bound"),
             rw(p + ".gamma_reparam.pedestal"), beta_eff, gamma_pk, gamma_eff, C, st);
    ConvW w;
    w.w = gamma_pk;
    w.b = beta_eff;
    w.Cin = w.Cout = C;
    w.K = 1;
    w.cin_pad = (C + 31) / 32 * 32;
    const int64_t nh = (int64_t)C * w.cin_pad;
    w.wh = reinterpret_cast<_Float16*>(take((nh + 1) / 2));
    w.wl = reinterpret_cast<_Float16*>(take((nh + 1) / 2));
    MLIC_CHECK(off <= total, "weight block");
    w.wexp = split_weights(gamma_eff, w.wh, w.wl, C, C, 1, w.cin_pad, true, st);
    w.name = p + ".__gdn";
    convs_[p + ".__gdn"] = w;
  }
  MLIC_CHECK(off <= total, "weight block overflow");
  // LDS-image copies for the x4 kernel: the stride-1 KxK convs it can serve (K in 1, 3, 5)
  {
    int64_t nx = 0;
    for (auto& kv : convs_) {
      const ConvW& w = kv.second;
      if (w.wh && (w.K == 1 || w.K == 3 || w.K == 5) && w.Cout >= 64) {
        nx += (x4_weight_halves(w.Cout, w.K * w.K, w.cin_pad) + 127) & ~(int64_t)127;
        if (gs_subpel(kv.first, w)) nx += (x4_weight_halves(w.Cout, w.K * w.K, w.cin_pad, true) + 127) & ~(int64_t)127;
      }
    }
    if (nx > 0) {
      _Float16* xb = nullptr;
      HIP_OK(hipMalloc(&xb, nx * sizeof(_Float16)));
      owned_.push_back(xb);
      wbytes_ += nx * sizeof(_Float16);
      int64_t xo = 0;
      for (auto& kv : convs_) {
        ConvW& w = kv.second;
        if (!(w.wh && (w.K == 1 || w.K == 3 || w.K == 5) && w.Cout >= 64)) continue;
        w.wx4 = xb + xo;
        x4_pack_weights(w.wh, w.wl, w.Cout, w.K * w.K, w.cin_pad, w.wx4, st);
        xo += (x4_weight_halves(w.Cout, w.K * w.K, w.cin_pad) + 127) & ~(int64_t)127;
        if (gs_subpel(kv.first, w)) {
          w.wx4h = xb + xo;
          x4_pack_weights(w.wh, w.wl, w.Cout, w.K * w.K, w.cin_pad, w.wx4h, st, true);
          xo += (x4_weight_halves(w.Cout, w.K * w.K, w.cin_pad, true) + 127) & ~(int64_t)127;
        }
      }
    }
  }
  // relative position index (attention.py:28-39), int32
  {
    const int win = cfg_.win, ww = win * win;
    std::vector<int> ri(ww * ww);
    for (int a = 0; a < ww; ++a)
      for (int c = 0; c < ww; ++c)
        ri[a * ww + c] = (a / win - c / win + win - 1) * (2 * win - 1) + (a % win - c % win + win - 1);
    rel_index_ = reinterpret_cast<int*>(take(ww * ww));
    HIP_OK(hipMemcpyAsync(rel_index_, ri.data(), ri.size() * 4, hipMemcpyHostToDevice, st));
  }
  add_chains(st);
  add_hoist(ep0, st);
  MLIC_CHECK(raw_.count("__scale_table"), "scale table missing");
  scale_table_ = const_cast<float*>(raw_["__scale_table"]);
  HIP_OK(hipStreamSynchronize(st));
}

// LocalContext's 5x5 fusion conv over the unfolded attention map (K index c*25 + cell, c = head*16 +
// d) as a conv_x4 GEMM over local_attn_packed's layout: K permuted to cell*32 + c, split, x4-packed
void Model::add_fusion_x4(const std::string& base, const float* w_dev, int Cout, hipStream_t st) {
  constexpr int CIN = 800;
  std::vector<float> w((size_t)Cout * CIN), wp((size_t)Cout * CIN);
  HIP_OK(hipMemcpyAsync(w.data(), w_dev, w.size() * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  for (int co = 0; co < Cout; ++co)
    for (int c = 0; c < 32; ++c)
      for (int cell = 0; cell < 25; ++cell) wp[(size_t)co * CIN + cell * 32 + c] = w[(size_t)co * CIN + c * 25 + cell];
  const int64_t nh = (int64_t)Cout * CIN, nx = x4_weight_halves(Cout, 1, CIN);
  char* blk = nullptr;
  const size_t bytes = (size_t)nh * 4 + 2 * (size_t)nh * 2 + (size_t)nx * 2 + 1024;
  HIP_OK(hipMalloc(&blk, bytes));
  owned_.push_back(blk);
  wbytes_ += bytes;
  float* wf = reinterpret_cast<float*>(blk);
  _Float16* wh = reinterpret_cast<_Float16*>(blk + (size_t)nh * 4);
  _Float16* wl = wh + nh;
  _Float16* wx = reinterpret_cast<_Float16*>((reinterpret_cast<uintptr_t>(wl + nh) + 255) & ~(uintptr_t)255);
  HIP_OK(hipMemcpyAsync(wf, wp.data(), wp.size() * 4, hipMemcpyHostToDevice, st));
  const int wexp = split_weights(wf, wh, wl, Cout, CIN, 1, CIN, true, st);
  x4_pack_weights(wh, wl, Cout, 1, CIN, wx, st);
  HIP_OK(hipStreamSynchronize(st));  // the host staging vectors die here
  ConvW cw;
  cw.w = wf;  // [Cout][800'] (not the fp32-MFMA packed layout: this ConvW only runs on conv_x4)
  cw.Cout = Cout;
  cw.Cin = CIN;
  cw.K = 1;
  cw.wh = wh;
  cw.wl = wl;
  cw.cin_pad = CIN;
  cw.wx4 = wx;
  cw.wexp = wexp;
  cw.name = base;
  convs_[base + ".__x4perm"] = cw;
}

// g_s's output conv (subpel_conv3x3(N, 3, 2): N -> 12, 3x3) as a 1x1 conv N -> 9 x 12 whose row
// tap * 12 + c holds w[c][:][tap]: the per-tap partial products, summed by taps_gather
void Model::add_taps(const std::string& base, const float* w_dev, int Cin, hipStream_t st) {
  constexpr int C = 12;
  std::vector<float> w((size_t)C * Cin * 9), wt((size_t)9 * C * Cin);
  HIP_OK(hipMemcpyAsync(w.data(), w_dev, w.size() * 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  for (int c = 0; c < C; ++c)
    for (int ci = 0; ci < Cin; ++ci)
      for (int t = 0; t < 9; ++t) wt[((size_t)t * C + c) * Cin + ci] = w[((size_t)c * Cin + ci) * 9 + t];
  float* tmp = nullptr;
  HIP_OK(hipMalloc(&tmp, wt.size() * 4));
  HIP_OK(hipMemcpyAsync(tmp, wt.data(), wt.size() * 4, hipMemcpyHostToDevice, st));
  convs_[base + ".__taps"] = make_conv(tmp, 9 * C, Cin, 1, base + ".__taps", st);
  HIP_OK(hipStreamSynchronize(st));
  HIP_OK(hipFree(tmp));
}

// $MLIC_TAPS=0: g_s's output conv on the narrow VALU kernel (A/B switch)
bool Model::taps_on() const {
  static const bool on = [] {
    const char* e = std::getenv("MLIC_TAPS");
    return !(e && std::atoi(e) == 0);
  }();
  return on && prec() == PREC_F16X3_V2;
}

// LDS weight images of the fused chains: EntropyParameters (entropy.py:10-18, layers .0 .2 .4 .6) and
// LocalContext's MLP (context.py:108-110, fc1 fc2)
void Model::add_chains(hipStream_t st) {
  std::vector<std::pair<std::string, std::vector<std::string>>> todo;
  for (auto& kv : convs_) {
    const std::string& k = kv.first;
    if (k.rfind("entropy_parameters", 0) == 0 && ends_with(k, ".fusion.0")) {
      const std::string p = k.substr(0, k.size() - 2);
      todo.push_back({p, {p + ".0", p + ".2", p + ".4", p + ".6"}});
    } else if (k.rfind("local_context", 0) == 0 && ends_with(k, ".mlp.fc1")) {
      const std::string p = k.substr(0, k.size() - 4);
      todo.push_back({p, {p + ".fc1", p + ".fc2"}});
    }
  }
  const int hyp = 2 * cfg_.hM();  // hyper_params channels: the last segment of every EP input
  int64_t total = 0;
  std::vector<ChainW> cws;
  for (auto& t : todo) {
    ChainW c;
    c.name = t.first;
    c.nl = (int)t.second.size();
    bool ok = true;
    for (int l = 0; l < c.nl; ++l) {
      auto it = convs_.find(t.second[l]);
      if (it == convs_.end() || it->second.K != 1 || !it->second.wh) { ok = false; break; }
      const ConvW& w = it->second;
      c.cout[l] = w.Cout;
      c.bias[l] = w.b;
      c.wexp[l] = w.wexp;
      if (l == 0) c.cin0 = w.Cin;
      else if (w.Cin != c.cout[l - 1]) ok = false;
      total += chain_layer_halves(w.Cout, w.Cin);
    }
    if (ok && chain_supported(c.nl, c.cout)) {
      if (c.cin0 % 64 == 0) cws.push_back(c);  // even K-step count (chain.hip)
      // the hoisted variant (context columns only) also serves EPs whose full input is an odd number of
      // 32-channel chunks (MLICPP_M_SMALL_DEC: 2 hM = 160 hyper channels)
      if (c.nl == 4 && c.cin0 >= hyp && (c.cin0 - hyp) % 64 == 0) {
        ChainW h = c;
        h.cin0 = c.cin0 - hyp;
        h.name = c.name + "#ctx";
        total += chain_layer_halves(c.cout[0], h.cin0);
        for (int l = 1; l < c.nl; ++l) total += chain_layer_halves(c.cout[l], c.cout[l - 1]);
        cws.push_back(h);
      }
    }
  }
  if (cws.empty()) return;
  _Float16* blk = nullptr;
  HIP_OK(hipMalloc(&blk, (size_t)total * sizeof(_Float16)));
  owned_.push_back(blk);
  wbytes_ += (size_t)total * sizeof(_Float16);
  int64_t off = 0;
  for (ChainW& c : cws) {
    c.wimg = blk + off;
    const bool ctx = ends_with(c.name, "#ctx");
    const std::string base = ctx ? c.name.substr(0, c.name.size() - 4) : c.name;
    const auto& names = c.nl == 4 ? std::vector<std::string>{base + ".0", base + ".2", base + ".4", base + ".6"}
                                  : std::vector<std::string>{base + ".fc1", base + ".fc2"};
    for (int l = 0; l < c.nl; ++l) {
      const ConvW& w = convs_.at(names[l]);
      const int cin = l == 0 ? c.cin0 : w.Cin;  // the hoisted variant packs the leading (context) columns
      if (cin > 0) chain_pack(w.wh, w.wl, w.Cout, cin, w.cin_pad, l > 0 ? 1 : 0, blk + off, st);
      off += chain_layer_halves(w.Cout, cin);
    }
    if (ctx) {
      c.name = base;
      chains_ctx_[base] = c;
    } else {
      chains_[c.name] = c;
    }
  }
}

// a standalone conv weight (the model's layer weights come from the state_dict loop above)
ConvW Model::make_conv(const float* w_dev, int Cout, int Cin, int K, const std::string& name, hipStream_t st) {
  ConvW w;
  w.Cout = Cout;
  w.Cin = Cin;
  w.K = K;
  w.cin_pad = (Cin + 31) / 32 * 32;
  w.name = name;
  const int64_t nw = (int64_t)Cout * Cin * K * K, nh = (int64_t)Cout * K * K * w.cin_pad;
  const int64_t nx = (K == 1 || K == 3 || K == 5) && Cout >= 64 ? x4_weight_halves(Cout, K * K, w.cin_pad) : 0;
  const size_t bytes = ((size_t)nw * 4 + 255) / 256 * 256 + 2 * (((size_t)nh * 2 + 255) / 256 * 256) + (size_t)nx * 2 + 256;
  char* blk = nullptr;
  HIP_OK(hipMalloc(&blk, bytes));
  owned_.push_back(blk);
  wbytes_ += bytes;
  w.w = reinterpret_cast<float*>(blk);
  w.wh = reinterpret_cast<_Float16*>(blk + ((size_t)nw * 4 + 255) / 256 * 256);
  w.wl = w.wh + ((size_t)nh * 2 + 255) / 256 * 256 / 2;
  pack_conv(w_dev, w.w, Cout, Cin, K * K, st);
  w.wexp = split_weights(w_dev, w.wh, w.wl, Cout, Cin, K * K, w.cin_pad, true, st);
  if (nx) {
    w.wx4 = w.wl + ((size_t)nh * 2 + 255) / 256 * 256 / 2;
    x4_pack_weights(w.wh, w.wl, Cout, K * K, w.cin_pad, w.wx4, st);
  }
  return w;
}

// EntropyParameters' layer 0 over [context..., hyper_params]: the hyper columns of all 2 S EPs stacked
// into one [2 S x C1][2 hM] weight (slot 2 i + nonanchor), so W_hyp . hyper is one GEMM per image
void Model::add_hoist(const std::map<std::string, std::pair<const float*, int>>& ep0, hipStream_t st) {
  const int hyp = 2 * cfg_.hM(), S = cfg_.S;
  if ((int)ep0.size() != 2 * S || chains_ctx_.size() != (size_t)(2 * S)) return;
  const int C1 = convs_.at("entropy_parameters_anchor.0.fusion.0").Cout;
  float* tmp = nullptr;
  HIP_OK(hipMalloc(&tmp, sizeof(float) * (size_t)2 * S * C1 * hyp));
  for (int i = 0; i < S; ++i)
    for (int k = 0; k < 2; ++k) {
      const std::string p = std::string("entropy_parameters_") + (k ? "nonanchor." : "anchor.") + std::to_string(i) +
                            ".fusion.0";
      auto it = ep0.find(p);
      MLIC_CHECK(it != ep0.end() && convs_.at(p).Cout == C1, "hoist: EP layer 0");
      const float* src = it->second.first;
      const int cin = it->second.second;
      HIP_OK(hipMemcpy2DAsync(tmp + (size_t)(2 * i + k) * C1 * hyp, (size_t)hyp * 4, src + (cin - hyp), (size_t)cin * 4,
                              (size_t)hyp * 4, C1, hipMemcpyDeviceToDevice, st));
    }
  hoist_ = make_conv(tmp, 2 * S * C1, hyp, 1, "__hyper_hoist", st);
  hoist_rows_ = C1;
  HIP_OK(hipStreamSynchronize(st));
  HIP_OK(hipFree(tmp));
}

// Whether EntropyParameters' hyper columns run as the one hoisted GEMM before the slice loop.  Default
// (auto): only when some EP's full input (context + hyper) cannot take the fused chain (an odd number of
// 32-channel chunks: MLICPP_M_SMALL_DEC's 2 hM = 160); otherwise every chain consumes hyper_params
// itself -- the chain kernel is VALU-bound with MFMA to spare, and the hoisted 640 -> 6400 GEMM costs
// ≈ 2 ms per 8 images on each side (measured, main config, alternating pairs on one box: 91.4 vs 89.9
// img/s).  $MLIC_HOIST=1 / 0 forces it on / off (A/B).
bool Model::hoist_on() const {
  static const int env = [] {
    const char* e = std::getenv("MLIC_HOIST");
    return e ? std::atoi(e) : -1;
  }();
  bool want = env >= 0 ? env != 0 : false;
  if (env < 0)
    for (int i = 0; i < cfg_.S && !want; ++i)
      for (const char* k : {"anchor", "nonanchor"})
        if (!chains_.count(std::string("entropy_parameters_") + k + "." + std::to_string(i) + ".fusion")) want = true;
  return want && chain_on() && hoist_.Cout > 0;
}

// the fused dwpw kernel (conv_dwpw.hip) instead of depthwise + resident pointwise for the stride-1
// dwsep convs with an even width (default; $MLIC_DWPW=0 is the A/B switch; the results are
// bit-identical either way)
bool Model::dwpw_on() const {
  static const bool on = [] {
    const char* e = std::getenv("MLIC_DWPW");
    return !(e && std::atoi(e) == 0);
  }();
  return on && prec() == PREC_F16X3_V2;
}

// $MLIC_CHAIN=0: the per-layer path for EntropyParameters / LocalContext MLP (A/B switch)
bool Model::chain_on() const {
  static const bool on = [] {
    const char* e = std::getenv("MLIC_CHAIN");
    return !(e && std::atoi(e) == 0);
  }();
  return on && prec() == PREC_F16X3_V2;
}

Model::~Model() {
  lanes_.clear();
  for (void* p : owned_) (void)hipFree(p);
}

Lane::~Lane() {
  if (rflag) (void)hipFree(rflag);
  for (void* p : {(void*)h_sym, (void*)h_sym16, (void*)h_idx8, (void*)hc_sym, (void*)hc_sym16, (void*)hc_idx8})
    if (p) (void)hipHostFree(p);
  if (cev) (void)hipEventDestroy(cev);
  if (cst) (void)hipStreamDestroy(cst);
  for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
  if (own_stream && st) (void)hipStreamDestroy(st);
}

thread_local Lane* Model::tl_lane_ = nullptr;

Lane& Model::lane(int i) {
  while ((int)lanes_.size() <= i) {
    auto l = std::make_unique<Lane>();
    // staggered priorities (lane 0 highest): symmetric lanes would reach their host entropy-coding
    // phases together and leave the GPU idle; with priorities they drift apart and each lane's host
    // coding overlaps the lower-priority lanes' kernels.  MLIC_LANE_PRIORITY=0 disables.
    const char* e = std::getenv("MLIC_LANE_PRIORITY");
    const bool stagger = !(e && std::atoi(e) == 0);
    if (stagger) {
      int least = 0, greatest = 0;
      HIP_OK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      const int prio = std::min(least, greatest + prio_base_ + (int)lanes_.size());
      HIP_OK(hipStreamCreateWithPriority(&l->st, hipStreamNonBlocking, prio));
    } else {
      HIP_OK(hipStreamCreateWithFlags(&l->st, hipStreamNonBlocking));
    }
    l->own_stream = true;
    l->prof = prof_;
    HIP_OK(hipMalloc(&l->rflag, sizeof(int)));
    HIP_OK(hipMemsetAsync(l->rflag, 0, sizeof(int), l->st));
    lanes_.push_back(std::move(l));
  }
  return *lanes_[i];
}

void Model::set_lanes(int n) {
  MLIC_CHECK(n >= 1 && n <= 16, "lanes must be in [1, 16]");
  nlanes_ = n;
}

void Model::set_profiling(bool on) {
  prof_ = on;
  for (auto& l : lanes_) l->prof = on;
}

size_t Model::arena_bytes() const {
  size_t s = 0;
  for (auto& l : lanes_) s += l->arena.capacity();
  return s;
}

const ConvW& Model::cw(const std::string& k) const {
  auto it = convs_.find(k);
  if (it == convs_.end()) throw Error("mlic: missing conv weight " + k);
  return it->second;
}
const DwW& Model::dww(const std::string& k) const {
  auto it = dws_.find(k);
  if (it == dws_.end()) throw Error("mlic: missing depthwise weight " + k);
  return it->second;
}
const float* Model::rw(const std::string& k) const {
  auto it = raw_.find(k);
  if (it == raw_.end()) throw Error("mlic: missing tensor " + k);
  return it->second;
}

// ------------------------------------------------------------------------------------- blocks
View Model::alloc(int C, int H, int W) {
  View v;
  v.p = L().arena.alloc((int64_t)L().B * C * H * W);
  v.C = C;
  v.H = H;
  v.W = W;
  v.bs = (int64_t)C * H * W;
  return v;
}

void Model::conv(const std::vector<View>& ins, const ConvW& w, int stride, int pad, const View& out, int epi,
                 const View* aux, const View* res) {
  const ConvParams P = conv_params(ins, w, stride, pad, out, epi, aux, res);
  run_conv(P, w, nullptr);
}

// two convs of one input (ResidualBlockUpsample's subpel_conv and upsample): on the x4 path the
// split-fp16 packing of the input is done once for both
void Model::conv_pair(const std::vector<View>& ins, const ConvW& w1, const View& out1, int epi1, const ConvW& w2,
                      const View& out2, int epi2) {
  const ConvParams P1 = conv_params(ins, w1, 1, w1.K / 2, out1, epi1, nullptr, nullptr);
  const ConvParams P2 = conv_params(ins, w2, 1, w2.K / 2, out2, epi2, nullptr, nullptr);
  const ConvWeights c1{w1.w, w1.wh, w1.wl, w1.cin_pad, w1.wx4, w1.wexp}, c2{w2.w, w2.wh, w2.wl, w2.cin_pad, w2.wx4, w2.wexp};
  if (conv_select(P1, c1, prec()) != CONV_X4 || conv_select(P2, c2, prec()) != CONV_X4 ||
      w1.cin_pad != w2.cin_pad || w1.K != w2.K) {
    run_conv(P1, w1, nullptr);
    run_conv(P2, w2, nullptr);
    return;
  }
  // the reduced-precision form when requested (set_synthesis_precision(1)) and both images exist
  const bool hi = gs_fp16_ && w1.wx4h && w2.wx4h;
  const size_t m = L().arena.mark();
  _Float16* act = reinterpret_cast<_Float16*>(L().arena.alloc((2 * x4_act_halves(P1, w1.cin_pad, hi) + 3) / 4));
  timed(PCAT_ELEM, 0.0, (hi ? 6.0 : 8.0) * L().B * P1.Cin * P1.H * P1.W,
        [&] { x4_pack_act(P1, w1.cin_pad, act, L().st, hi); }, w1.name + ".__x4_pack");
  run_conv(P1, w1, act, hi);
  run_conv(P2, w2, act, hi);
  L().arena.release(m);
}

// packed: the input already in x4's split layout (conv_pair); the impl is then necessarily x4
void Model::run_conv(const ConvParams& P, const ConvW& w, const _Float16* packed, bool hi, bool split) {
  const ConvWeights cw{w.w, w.wh, w.wl, w.cin_pad, w.wx4, w.wexp};
  const int impl = packed ? (hi ? CONV_X4H : CONV_X4) : conv_select(P, cw, prec());
  const double outn = (double)P.B * w.Cout * P.Ho * P.Wo;
  const double flops = 2.0 * outn * P.Cin * w.K * w.K;
  const double bytes = 4.0 * ((double)P.B * P.Cin * P.H * P.W + (double)w.Cout * P.Cin * w.K * w.K +
                              outn * (1 + (P.aux ? 1 : 0) + (P.res ? 1 : 0)));
  // profile tag: layer name + shape (Cin>Cout kK sS, epilogue flags, input segments)
  std::string tag;
  if (L().prof) {
    char sh[96];
    std::snprintf(sh, sizeof sh, " [%d>%d k%d s%d e%x n%d]", P.Cin, P.Cout, P.K, P.stride, P.epi, P.nseg);
    tag = w.name + sh;
  }
  if (packed) {
    // split: the few-tile split-K path of conv_run (x4_splitk), for a packed operand made elsewhere
    const int64_t pb = split ? x4_part_bytes(P, w.cin_pad, hi) : 0;
    const size_t m = L().arena.mark();
    float* part = pb > 0 ? L().arena.alloc((pb + 3) / 4) : nullptr;
    timed(conv_prof_cat(impl, P), flops, bytes,
          [&] { conv_x4_forward(P, packed, hi ? w.wx4h : w.wx4, w.cin_pad, L().st, part, hi); }, tag);
    L().arena.release(m);
    return;
  }
  const int64_t wsb = conv_ws_bytes(impl, P, cw);
  const size_t m = L().arena.mark();
  void* ws = wsb > 0 ? static_cast<void*>(L().arena.alloc((wsb + 3) / 4)) : nullptr;
  timed(conv_prof_cat(impl, P), flops, bytes, [&] { conv_run(impl, P, cw, L().st, ws); }, tag);
  L().arena.release(m);  // stream-ordered: the next user of this memory runs after the conv
}

ConvParams Model::conv_params(const std::vector<View>& ins, const ConvW& w, int stride, int pad, const View& out,
                              int epi, const View* aux, const View* res) {
  ConvParams P{};
  MLIC_CHECK(!ins.empty() && (int)ins.size() <= MAXSEG, "conv inputs");
  P.nseg = (int)ins.size();
  int cin = 0;
  for (int s = 0; s < P.nseg; ++s) {
    MLIC_CHECK(ins[s].H == ins[0].H && ins[s].W == ins[0].W, "concat inputs must share H, W");
    P.seg[s] = {ins[s].p, ins[s].C, ins[s].bs};
    cin += ins[s].C;
  }
  MLIC_CHECK(cin == w.Cin, "conv Cin mismatch");
  P.Cin = cin;
  P.H = ins[0].H;
  P.W = ins[0].W;
  P.Cout = w.Cout;
  P.K = w.K;
  P.stride = stride;
  P.pad = pad;
  P.Ho = (P.H + 2 * pad - w.K) / stride + 1;
  P.Wo = (P.W + 2 * pad - w.K) / stride + 1;
  P.wpk = w.w;
  P.wexp = w.wexp;  // conv_run clears it for the fp32 families
  P.rflag = L().rflag;
  P.bias = w.b;
  P.epi = epi;
  if (epi & EPI_SHUFFLE) {
    MLIC_CHECK(out.C * 4 == w.Cout && out.H == 2 * P.Ho && out.W == 2 * P.Wo, "shuffle output shape");
  } else {
    MLIC_CHECK(out.C == w.Cout && out.H == P.Ho && out.W == P.Wo, "conv output shape");
  }
  P.out = out.p;
  P.out_bs = out.bs;
  P.out_cs = out.hw();
  if (aux) {
    MLIC_CHECK(aux->C == w.Cout && aux->H == P.Ho && aux->W == P.Wo, "aux shape");
    P.aux = aux->p;
    P.aux_bs = aux->bs;
  }
  if (res) {
    MLIC_CHECK(res->C == out.C && res->H == out.H && res->W == out.W, "residual shape");
    P.res = res->p;
    P.res_bs = res->bs;
    P.epi |= EPI_RES;
  }
  P.B = L().B;
  return P;
}

void Model::dw(const std::vector<View>& ins, const DwW& w, int stride, const View& out, bool gelu) {
  DwParams P{};
  P.nseg = (int)ins.size();
  int c = 0;
  for (int s = 0; s < P.nseg; ++s) {
    P.seg[s] = {ins[s].p, ins[s].C, ins[s].bs};
    c += ins[s].C;
  }
  MLIC_CHECK(c == w.C && out.C == w.C, "depthwise channels");
  P.C = c;
  P.H = ins[0].H;
  P.W = ins[0].W;
  P.stride = stride;
  P.Ho = (P.H - 1) / stride + 1;
  P.Wo = (P.W - 1) / stride + 1;
  MLIC_CHECK(out.H == P.Ho && out.W == P.Wo, "depthwise output shape");
  P.w = w.w;
  P.bias = w.b;
  P.out = out.p;
  P.out_bs = out.bs;
  P.gelu = gelu ? 1 : 0;
  P.B = L().B;
  const double outn = (double)L().B * c * P.Ho * P.Wo;
  timed(PCAT_DW, 18.0 * outn, 4.0 * ((double)L().B * c * P.H * P.W + outn), [&] { dw3x3(P, L().st); }, w.name);
}

// a fused chain over a (multi-segment) input; GELU between the layers (entropy.py:10-18, MLP fc1 -> fc2)
void Model::run_chain(const ChainW& c, const std::vector<View>& ins, const View& out, const View* res,
                      const View* aux, int H, int W, int ckbd, bool sq_in) {
  ChainParams P{};
  MLIC_CHECK((int)ins.size() <= MAXSEG && (!ins.empty() || aux), "chain inputs");
  if (!ins.empty()) {
    H = ins[0].H;
    W = ins[0].W;
  }
  P.nseg = (int)ins.size();
  int cin = 0;
  for (int s = 0; s < P.nseg; ++s) {
    MLIC_CHECK(ins[s].H == H && ins[s].W == W, "chain inputs must share H, W");
    P.seg[s] = {ins[s].p, ins[s].C, ins[s].bs};
    cin += ins[s].C;
  }
  MLIC_CHECK(cin == c.cin0, "chain Cin mismatch");
  MLIC_CHECK(!sq_in || (ckbd && !aux), "chain: squeezed inputs need a checkerboard half");
  if (sq_in) W *= 2;  // squeezed input planes (H x W / 2): the output is the full grid
  MLIC_CHECK(out.C == c.cout[c.nl - 1] && out.H == H && out.W == W, "chain output shape");
  if (aux) {
    MLIC_CHECK(aux->C == c.cout[0] && aux->H == H && aux->W == W, "chain aux shape");
    P.aux = aux->p;
    P.aux_bs = aux->bs;
  }
  P.cin0 = cin;
  P.HW = H * W;
  P.W = W;
  P.ckbd = ckbd;
  P.sq_in = sq_in ? 1 : 0;
  P.B = L().B;
  for (int l = 0; l < 4; ++l) {
    P.bias[l] = c.bias[l];
    P.wexp[l] = c.wexp[l];
  }
  P.wimg = c.wimg;
  P.rflag = L().rflag;
  P.out = out.p;
  P.out_bs = out.bs;
  if (res) {
    MLIC_CHECK(res->C == out.C && res->H == out.H && res->W * (sq_in ? 2 : 1) == out.W, "chain residual shape");
    P.res = res->p;
    P.res_bs = res->bs;
  }
  double mac = (double)c.cin0 * c.cout[0];
  for (int l = 1; l < c.nl; ++l) mac += (double)c.cout[l - 1] * c.cout[l];
  const double pix = (double)P.B * (ckbd ? P.HW / 2 : P.HW);
  const double bytes = 4.0 * (pix * (cin + out.C * (res ? 2 : 1) + (aux ? c.cout[0] : 0)) + mac);
  timed(PCAT_CHAIN, 2.0 * mac * pix, bytes, [&] { chain_forward(P, c.nl, c.cout, L().st); }, c.name);
}

// conv3x3 of the fork (modules/layers/conv.py:22-32): DepthWiseConv (dw 3x3 -> pw 1x1) by default,
// compressai's dense 3x3 for the *_old modules.  `epi` applies to the last (pointwise) conv.
View Model::conv3x3(const std::vector<View>& ins, const std::string& p, int stride, bool dwsep, int epi,
                    const View* res, const View* out_opt) {
  const int H = ins[0].H, W = ins[0].W;
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  if (!dwsep) {
    const ConvW& w = cw(p);
    View out = out_opt ? *out_opt : alloc(w.Cout, Ho, Wo);
    conv(ins, w, stride, 1, out, epi, nullptr, res);
    return out;
  }
  const DwW& d = dww(p + ".depth_conv");
  const ConvW& w = cw(p + ".point_conv");
  View out = out_opt ? *out_opt : alloc(w.Cout, Ho, Wo);
  if (stride == 1 && dwpw_on() && w.wh && ins.size() == 1) {
    // fused: the pointwise conv reads the depthwise input; the depthwise output stays on chip
    ConvParams P = conv_params(ins, w, 1, 0, out, epi, nullptr, res);
    if (dwpw_ok(P, w.cin_pad) && dwpw_grid_ok(P)) {
      const double pix = (double)P.B * H * W;
      const double flops = 2.0 * pix * P.Cin * (9 + w.Cout);
      const double bytes = 4.0 * (pix * (P.Cin + w.Cout * (res ? 2 : 1)) + (double)w.Cout * P.Cin + 10.0 * P.Cin);
      timed(PCAT_DWPW, flops, bytes, [&] { dwpw_forward(P, w.wh, w.wl, w.cin_pad, d.w, d.b, L().st); }, w.name);
      return out;
    }
  }
  const size_t m = L().arena.mark();
  View t = alloc(d.C, Ho, Wo);
  dw(ins, d, stride, t, false);
  conv({t}, w, 1, 0, out, epi, nullptr, res);
  L().arena.release(m);
  return out;
}

View Model::conv1x1(const View& in, const std::string& p, int stride, int epi, const View* res) {
  const ConvW& w = cw(p);
  View out = alloc(w.Cout, (in.H - 1) / stride + 1, (in.W - 1) / stride + 1);
  conv({in}, w, stride, 0, out, epi, nullptr, res);
  return out;
}

// compressai GDN: out = x * rsqrt(conv2d(x^2, gamma, beta)) (inverse: * sqrt)
void Model::gdn(const View& x, const std::string& p, bool inverse, const View& out, const View* res) {
  conv({x}, cw(p + ".__gdn"), 1, 0, out, EPI_SQUARE_IN | (inverse ? EPI_IGDN : EPI_GDN), &x, res);
}

// res_blk.py:62-93 ResidualBlockWithStride
View Model::rbws(const View& x, const std::string& p, bool dwsep) {
  const int Ho = (x.H - 1) / 2 + 1, Wo = (x.W - 1) / 2 + 1;
  const ConvW& sk = cw(p + ".skip");
  View out = alloc(sk.Cout, Ho, Wo);
  const size_t m = L().arena.mark();
  View t1 = conv3x3({x}, p + ".conv1", 2, dwsep, EPI_GELU);
  View t2 = conv3x3({t1}, p + ".conv2", 1, dwsep, EPI_NONE);
  View s = alloc(sk.Cout, Ho, Wo);
  conv({x}, sk, 2, 0, s, EPI_NONE);
  gdn(t2, p + ".gdn", false, out, &s);
  L().arena.release(m);
  return out;
}

// res_blk.py:124-154 ResidualBlock: out = gelu(conv2(gelu(conv1(x)))) + (skip(x) or x)
View Model::rb(const View& x, const std::string& p, bool dwsep) {
  const bool has_skip = convs_.count(p + ".skip") > 0;
  const int Cout = dwsep ? cw(p + ".conv2.point_conv").Cout : cw(p + ".conv2").Cout;
  View out = alloc(Cout, x.H, x.W);
  const size_t m = L().arena.mark();
  View t1 = conv3x3({x}, p + ".conv1", 1, dwsep, EPI_GELU);
  View id = x;
  if (has_skip) {
    id = alloc(Cout, x.H, x.W);
    conv({x}, cw(p + ".skip"), 1, 0, id, EPI_NONE);
  }
  conv3x3({t1}, p + ".conv2", 1, dwsep, EPI_GELU, &id, &out);
  L().arena.release(m);
  return out;
}

// res_blk.py:96-121 ResidualBlockUpsample: igdn(dwsep(gelu(subpel(x)))) + subpel_up(x)
View Model::rbu(const View& x, const std::string& p) {
  const ConvW& a = cw(p + ".subpel_conv.0");
  const ConvW& u = cw(p + ".upsample.0");
  const int C = a.Cout / 4;
  View out = alloc(C, 2 * x.H, 2 * x.W);
  const size_t m = L().arena.mark();
  View ta = alloc(C, 2 * x.H, 2 * x.W);
  View tu = alloc(C, 2 * x.H, 2 * x.W);
  conv_pair({x}, a, ta, EPI_GELU | EPI_SHUFFLE, u, tu, EPI_SHUFFLE);
  View tc = conv3x3({ta}, p + ".conv", 1, true, EPI_NONE);
  gdn(tc, p + ".igdn", true, out, &tu);
  L().arena.release(m);
  return out;
}

// analysis.py:6-22 (SD: analysis_old with dense 3x3)
View Model::g_a(const View& x) {
  const bool dwsep = !cfg_.sd;
  const std::string g = "g_a.analysis_transform";
  const int M = cfg_.M;
  View y = alloc(M, (x.H + 15) / 16, (x.W + 15) / 16);
  const size_t m = L().arena.mark();
  View a = rbws(x, g + ".0", dwsep);
  View b = rb(a, g + ".1", dwsep);
  View c = rbws(b, g + ".2", dwsep);
  View d = rb(c, g + ".3", dwsep);
  View e = rbws(d, g + ".4", dwsep);
  View f = rb(e, g + ".5", dwsep);
  conv3x3({f}, g + ".6", 2, dwsep, EPI_NONE, nullptr, &y);
  L().arena.release(m);
  return y;
}

// analysis.py:25-48
View Model::h_a(const View& y) {
  const bool dwsep = !cfg_.sd;
  const std::string h = "h_a.reduction";
  View z = alloc(cfg_.N, (y.H + 3) / 4, (y.W + 3) / 4);
  const size_t m = L().arena.mark();
  View a = conv3x3({y}, h + ".0", 1, dwsep, EPI_GELU);
  View b = conv3x3({a}, h + ".2", 1, dwsep, EPI_GELU);
  View c = conv3x3({b}, h + ".4", 2, dwsep, EPI_GELU);
  View d = conv3x3({c}, h + ".6", 1, dwsep, EPI_GELU);
  conv3x3({d}, h + ".8", 2, dwsep, EPI_NONE, nullptr, &z);
  L().arena.release(m);
  return z;
}

// synthesis.py:9-33
View Model::h_s(const View& z) {
  const std::string h = "h_s.increase";
  const int hM = cfg_.hM();
  View out = alloc(2 * hM, 4 * z.H, 4 * z.W);
  const size_t m = L().arena.mark();
  View a = conv3x3({z}, h + ".0", 1, true, EPI_GELU);
  View b = alloc(hM, 2 * z.H, 2 * z.W);
  conv({a}, cw(h + ".2.0"), 1, 1, b, EPI_GELU | EPI_SHUFFLE);
  View c = conv3x3({b}, h + ".4", 1, true, EPI_GELU);
  View d = alloc(hM * 3 / 2, 4 * z.H, 4 * z.W);
  conv({c}, cw(h + ".6.0"), 1, 1, d, EPI_GELU | EPI_SHUFFLE);
  conv3x3({d}, h + ".8", 1, true, EPI_NONE, nullptr, &out);
  L().arena.release(m);
  return out;
}

// synthesis.py:56-73
void Model::g_s(const View& yh, const View& out) {
  const std::string g = "g_s.synthesis_transform";
  const size_t m = L().arena.mark();
  View a = rb(yh, g + ".0", true);
  View b = rbu(a, g + ".1");
  View c = rb(b, g + ".2", true);
  View d = rbu(c, g + ".3");
  View e = rb(d, g + ".4", true);
  View f = rbu(e, g + ".5");
  View h = rb(f, g + ".6", true);
  auto tp = convs_.find(g + ".7.0.__taps");
  const ConvW& w7 = cw(g + ".7.0");
  if (tp != convs_.end() && taps_on()) {
    // per-tap partials on the resident 1x1 kernel, then the fixed-order tap sum + bias + shuffle
    const size_t m2 = L().arena.mark();
    View part = alloc(tp->second.Cout, h.H, h.W);
    conv({h}, tp->second, 1, 0, part, EPI_NONE);
    const double pix = (double)L().B * h.H * h.W;
    timed(PCAT_CONV_NARROW, pix * 9 * 12, 4.0 * pix * (9 * 12 + 12), [&] {
      taps_gather(part.p, part.bs, w7.b, out.p, out.bs, h.H, h.W, L().B, L().st);
    }, g + ".7.0.__gather");
    L().arena.release(m2);
  } else {
    conv({h}, w7, 1, 1, out, EPI_SHUFFLE);
  }
  L().arena.release(m);
}

// ------------------------------------------------------------------------------------- MEM++
// context.py:67-112 LocalContext
View Model::local_context(const View& x, int i, bool half) {
  const std::string p = "local_context." + std::to_string(i);
  const int C = x.C, H = x.H, W = x.W;
  View out = alloc(2 * C, H, W);
  const size_t m = L().arena.mark();
  static const bool packed_on = [] {  // $MLIC_LA_PACKED=0: the unfolded fp32 path (A/B switch)
    const char* e = std::getenv("MLIC_LA_PACKED");
    return !(e && std::atoi(e) == 0);
  }();
  const bool packed = packed_on && prec() == PREC_F16X3_V2 && C == 32 && convs_.count(p + ".fusion.__x4perm");
  // non-anchor half only: every stage after the qkv projection is per query pixel, so it runs on the
  // squeezed half (planes of H x W / 2, pixel y W / 2 + x / 2) and the MLP chain writes the full-grid
  // output at the non-anchor pixels (the reference computes the whole grid; its only consumer, the
  // non-anchor EntropyParameters, reads these pixels: mlicpp.py:237-241, 267-271)
  auto cit = chains_.find(p + ".mlp");
  half = half && packed && W % 2 == 0 && chain_on() && cit != chains_.end() && (H * W) % 8 == 0;
  const int Wq = half ? W / 2 : W;
  View n1 = alloc(C, H, W);
  const double pix = (double)L().B * H * W;
  timed(PCAT_ELEM, 8.0 * pix * C, 8.0 * pix * C, [&] {
    ln_channels(x.p, x.bs, n1.p, n1.bs, rw(p + ".norm1.weight"), rw(p + ".norm1.bias"), C, H * W, L().B, L().st);
  }, p + ".norm1");
  View qkv = conv1x1(n1, p + ".qkv_proj", 1, EPI_NONE);
  View f = alloc(2 * C, H, Wq);
  if (packed) {
    // attention straight into the fusion conv's packed split operand, fusion on conv_x4
    const ConvW& fw = cw(p + ".fusion.__x4perm");
    const int npos = (H * Wq + 31) / 32 * 32;
    _Float16* tp = reinterpret_cast<_Float16*>(L().arena.alloc((int64_t)L().B * 25 * npos * 32));
    LocalAttnParams A{};
    A.qkv = qkv.p;
    A.qkv_bs = qkv.bs;
    A.rel_table = rw(p + ".relative_position_table");
    A.rel_index = rel_index_;
    A.scale = (float)std::pow((double)(C / 2), -0.5);  // context.py:27 head_dim ** -0.5
    A.C = C;
    A.H = H;
    A.W = W;
    A.B = L().B;
    A.ckbd = half ? 2 : 0;
    const double fl = (half ? 0.5 : 1.0) * pix * 2.0 * 2 * 25 * 25 * (C / 2) * 2;
    timed(PCAT_LOCAL, fl, 4.0 * pix * (3 * C + (half ? 0.5 : 1.0) * 25 * C), [&] { local_attn_packed(A, tp, npos, L().st); },
          p + ".attn");
    const View tv{nullptr, 25 * C, H, Wq, (int64_t)25 * C * H * Wq};  // geometry only: conv_x4 reads tp
    run_conv(conv_params({tv}, fw, 1, 0, f, EPI_NONE, nullptr, nullptr), fw, tp);
  } else {
  View t = alloc(25 * C, H, W);
  {
    LocalAttnParams A{};
    A.qkv = qkv.p;
    A.qkv_bs = qkv.bs;
    A.out = t.p;
    A.out_bs = t.bs;
    A.rel_table = rw(p + ".relative_position_table");
    A.rel_index = rel_index_;
    A.scale = (float)std::pow((double)(C / 2), -0.5);  // context.py:27 head_dim ** -0.5
    A.C = C;
    A.H = H;
    A.W = W;
    A.B = L().B;
    // per pixel: 2 heads x 25 query cells x 25 keys x hd (QK) + the same for AV
    const double fl = pix * 2.0 * 2 * 25 * 25 * (C / 2) * 2;
    timed(PCAT_LOCAL, fl, 4.0 * pix * (3 * C + 25 * C), [&] { local_attn(A, L().st); }, p + ".attn");
  }
  conv({t}, cw(p + ".fusion"), 1, 0, f, EPI_NONE);
  }
  View pj = conv1x1(f, p + ".proj", 1, EPI_NONE);
  View n2 = alloc(2 * C, H, Wq);
  const double pq = (double)L().B * H * Wq;
  timed(PCAT_ELEM, 16.0 * pq * C, 16.0 * pq * C, [&] {
    ln_channels(pj.p, pj.bs, n2.p, n2.bs, rw(p + ".norm2.weight"), rw(p + ".norm2.bias"), 2 * C, H * Wq, L().B, L().st);
  }, p + ".norm2");
  auto ch = cit;
  if (half) {
    run_chain(ch->second, {n2}, out, &pj, nullptr, 0, 0, 2, true);
  } else if (chain_on() && ch != chains_.end() && (H * W) % 4 == 0) {
    run_chain(ch->second, {n2}, out, &pj);
  } else {
    View h1 = conv1x1(n2, p + ".mlp.fc1", 1, EPI_GELU);
    conv({h1}, cw(p + ".mlp.fc2"), 1, 0, out, EPI_NONE, nullptr, &pj);
  }
  L().arena.release(m);
  return out;
}

// context.py:115-138 ChannelContext (SD: context_old, dense 3x3)
View Model::channel_context(const View& x, int i) {
  const std::string p = "channel_context." + std::to_string(i) + ".fushion";
  const bool dwsep = !cfg_.sd;
  const int Cout = dwsep ? cw(p + ".4.point_conv").Cout : cw(p + ".4").Cout;
  View out = alloc(Cout, x.H, x.W);
  const size_t m = L().arena.mark();
  View a = conv3x3({x}, p + ".0", 1, dwsep, EPI_GELU);
  View b = conv3x3({a}, p + ".2", 1, dwsep, EPI_GELU);
  conv3x3({b}, p + ".4", 1, dwsep, EPI_NONE, nullptr, &out);
  L().arena.release(m);
  return out;
}

// nn.Sequential(conv1x1, depthwise 3x3) of keys/queries/values
View Model::qkv_branch(const View& x, const std::string& p) {
  const DwW& d = dww(p + ".1");
  View out = alloc(d.C, x.H, x.W);
  const size_t m = L().arena.mark();
  View t = conv1x1(x, p + ".0", 1, EPI_NONE);
  dw({t}, d, 1, out, false);
  L().arena.release(m);
  return out;
}

static int ctx_splits(int HW) { return std::max(1, std::min(64, HW / 256)); }

// context.py:195-245 LinearGlobalInterContext
View Model::inter_context(const View& x, int i) {
  const std::string p = "global_inter_context." + std::to_string(i);
  const int D = x.C, H = x.H, W = x.W, HW = H * W;
  const int heads = D / 32, hd = 32;  // num_heads = slice_ch * i // 32 (mlicpp.py:50)
  const ConvW& sk = cw(p + ".skip");
  View out = alloc(sk.Cout, H, W);
  const size_t m = L().arena.mark();
  View q = qkv_branch(x, p + ".queries");
  View k = qkv_branch(x, p + ".keys");
  View v = qkv_branch(x, p + ".values");
  const ConvW& rp = cw(p + ".reprojection");
  View a = alloc(rp.Cout, H, W);
  linatt_reproject(k, v, q, heads, hd, 0, 0, rp, a, p + ".attn");
  View m1 = conv1x1(a, p + ".mlp.0", 1, EPI_GELU);
  View m2 = alloc(m1.C, H, W);
  dw({m1}, dww(p + ".mlp.2"), 1, m2, true);
  View s = conv1x1(a, p + ".skip", 1, EPI_NONE);
  conv({m2}, cw(p + ".mlp.4"), 1, 0, out, EPI_NONE, nullptr, &s);
  L().arena.release(m);
  return out;
}

// $MLIC_LINATT_FUSED=0: the three-launch linear attention + fp32 att + the reprojection's own pack (A/B)
static int g_linatt_fused = -1;  // mlic_set_kernel_option("linatt_fused"): -1 = the environment / on
void linatt_set_fused(int on) { g_linatt_fused = on; }
static bool linatt_fused_on() {
  static const bool env = [] {
    const char* e = std::getenv("MLIC_LINATT_FUSED");
    return !(e && std::atoi(e) == 0);
  }();
  return g_linatt_fused < 0 ? env : g_linatt_fused != 0;
}

// the linear attention and the 5x5 reprojection conv that consumes it (context.py:180-190, 235-241).
// Fused (default, when the reprojection runs on conv_x4): ctx (partials + the fixed-order combine),
// then ctx^T . softmax_c(q) written straight into the conv's packed split operand -- the fp32
// attention map is never stored and the conv's own packing pass is gone.  Bit-identical to the
// unfused form (linatt_pack_kernel).
void Model::linatt_reproject(const View& k, const View& v, const View& q, int heads, int hd, int kmask, int qmask,
                             const ConvW& rp, const View& a, const std::string& tag) {
  const int H = q.H, W = q.W, HW = H * W, D = heads * hd, B = L().B;
  const int nsplit = ctx_splits(HW);
  const size_t m = L().arena.mark();
  float* part = L().arena.alloc(linear_attention_part_floats(heads, hd, B, nsplit));
  float* ctx = L().arena.alloc((int64_t)B * heads * hd * hd);
  // algorithmic bytes: k, v, q read once, the attention written once
  const double fl = (double)B * HW * D * hd * 4.0, by = 4.0 * B * HW * D * 4.0;
  const View geo{nullptr, D, H, W, (int64_t)D * HW};  // geometry only: the fused conv reads its packed operand
  const ConvParams P = conv_params({geo}, rp, 1, 2, a, EPI_NONE, nullptr, nullptr);
  const ConvWeights cwt{rp.w, rp.wh, rp.wl, rp.cin_pad, rp.wx4, rp.wexp};
  if (linatt_fused_on() && rp.cin_pad == D && D % 32 == 0 && conv_select(P, cwt, prec()) == CONV_X4) {
    timed(PCAT_LINATT, fl * 0.5, 4.0 * B * HW * D * 2.0, [&] {
      linear_attention_ctx(k.p, k.bs, v.p, v.bs, part, ctx, heads, hd, H, W, B, nsplit, kmask, L().st);
    }, tag);
    _Float16* act = reinterpret_cast<_Float16*>(L().arena.alloc((2 * x4_act_halves(P, rp.cin_pad) + 3) / 4));
    timed(PCAT_LINATT, fl * 0.5, 4.0 * B * HW * D * 2.0, [&] {
      linatt_pack(q.p, q.bs, ctx, heads, hd, qmask, P, act, L().st);
    }, tag + ".pack");
    run_conv(P, rp, act, false, true);
  } else {
    View att = alloc(D, H, W);
    timed(PCAT_LINATT, fl, by, [&] {
      linear_attention(k.p, k.bs, v.p, v.bs, q.p, q.bs, att.p, att.bs, part, ctx, heads, hd, H, W, B, nsplit, kmask, qmask,
                       L().st);
    }, tag);
    conv({att}, rp, 1, 2, a, EPI_NONE);
  }
  L().arena.release(m);
}

// context.py:140-193 LinearGlobalIntraContext: q from non-anchor cells of x1, k from anchor cells of
// x1, v from x2; the squeezed-half softmaxes are computed on the full grid with parity masks.
View Model::intra_context(const View& x1, const View& x2, int i) {
  const std::string p = "global_intra_context." + std::to_string(i);
  const int D = x1.C, H = x1.H, W = x1.W, HW = H * W;
  const int heads = 2, hd = D / 2;
  View out = alloc(2 * D, H, W);
  const size_t m = L().arena.mark();
  View x1n = alloc(D, H, W);
  View x1a = alloc(D, H, W);
  timed(PCAT_ELEM, 0.0, 16.0 * L().B * D * HW, [&] {
    ckbd_mask(x1.p, x1.bs, x1n.p, x1n.bs, D, H, W, L().B, 0, L().st);
    ckbd_mask(x1.p, x1.bs, x1a.p, x1a.bs, D, H, W, L().B, 1, L().st);
  }, p + ".ckbd");
  View q = qkv_branch(x1n, p + ".queries");
  View k = qkv_branch(x1a, p + ".keys");
  View v = qkv_branch(x2, p + ".values");
  const ConvW& rp = cw(p + ".reprojection");
  View a = alloc(rp.Cout, H, W);
  linatt_reproject(k, v, q, heads, hd, 1, 2, rp, a, p + ".attn");
  View m1 = conv1x1(a, p + ".mlp.0", 1, EPI_GELU);
  View m2 = alloc(m1.C, H, W);
  dw({m1}, dww(p + ".mlp.2"), 1, m2, true);
  conv({m2}, cw(p + ".mlp.4"), 1, 0, out, EPI_NONE, nullptr, &a);
  L().arena.release(m);
  return out;
}

// entropy.py:7-29
bool Model::ep_half_chain(const std::string& kind, int i, int H, int W, bool hoisted) const {
  const std::string p = "entropy_parameters_" + kind + "." + std::to_string(i) + ".fusion";
  if (!chain_ep_half() || W % 2 != 0 || (H * W) % 4 != 0) return false;
  return hoisted ? chains_ctx_.count(p) > 0 : (chain_on() && chains_.count(p) > 0);
}

View Model::entropy_parameters(const std::vector<View>& ctx, const View* hyper, const std::string& kind, int i,
                               const View* hoisted, bool phase_only) {
  const std::string p = "entropy_parameters_" + kind + "." + std::to_string(i) + ".fusion";
  const View& geo = ctx.empty() ? *hyper : ctx[0];
  const int H = geo.H, W = geo.W;
  // the phase's checkerboard half only: the reference computes the whole grid and masks the other half
  // to zero (ckbd_anchor / ckbd_nonanchor, mlicpp.py:226-228, 239-241) before any use
  const int ckbd = phase_only && chain_ep_half() && W % 2 == 0 ? (kind == "nonanchor" ? 2 : 1) : 0;
  const ConvW& l3 = cw(p + ".6");
  View out = alloc(l3.Cout, H, W);
  auto hc = chains_ctx_.find(p);
  if (hoisted && hc != chains_ctx_.end() && (H * W) % 4 == 0) {
    const int slot = 2 * i + (kind == "nonanchor" ? 1 : 0);
    const View aux = hoisted->ch(slot * hoist_rows_, hoist_rows_);
    run_chain(hc->second, ctx, out, nullptr, &aux, H, W, ckbd);
    return out;
  }
  std::vector<View> ins = ctx;
  if (hyper) ins.push_back(*hyper);
  auto ch = chains_.find(p);
  if (chain_on() && ch != chains_.end() && (H * W) % 4 == 0) {
    run_chain(ch->second, ins, out, nullptr, nullptr, 0, 0, ckbd);
    return out;
  }
  const size_t m = L().arena.mark();
  View a = alloc(cw(p + ".0").Cout, H, W);
  conv(ins, cw(p + ".0"), 1, 0, a, EPI_GELU);
  View b = conv1x1(a, p + ".2", 1, EPI_GELU);
  View c = conv1x1(b, p + ".4", 1, EPI_GELU);
  conv({c}, l3, 1, 0, out, EPI_NONE);
  L().arena.release(m);
  return out;
}

// quantization.py:30-44 (SD: LatentResidualPredictionOld, 4 layers); the last conv's epilogue
// applies 0.5*tanh, the checkerboard mask and the residual add into the y_hat slice in place
// (mlicpp.py:119-120, 137-138).
void Model::lrp(const std::vector<View>& ins, const std::string& kind, int i, const View& yh, bool anchor) {
  const std::string p = "lrp_" + kind + "." + std::to_string(i) + ".lrp_transform";
  const int nl = cfg_.sd ? 4 : 3;
  const size_t m = L().arena.mark();
  std::vector<View> cur = ins;
  for (int l = 0; l < nl; ++l) {
    const std::string q = p + "." + std::to_string(2 * l);
    if (l + 1 < nl) {
      View o = conv3x3(cur, q, 1, true, EPI_GELU);
      cur = {o};
    } else {
      const int epi = EPI_TANH_HALF | (anchor ? EPI_MASK_ANCHOR : EPI_MASK_NONANCHOR);
      conv3x3(cur, q, 1, true, epi, &yh, &yh);
    }
  }
  L().arena.release(m);
}

// ------------------------------------------------------------------------------------- phases
class PhaseDecoder {
 public:
  // single: y[0] holds every image's symbols, phase-major then image-minor (the reference's batched
  // stream); one decoder then walks the images of each phase in order
  PhaseDecoder(int B, const uint8_t* const* y, const size_t* ylen, const CdfTables* t, int32_t* h_sym,
               int16_t* h_sym16, uint8_t* h_idx8, HostStats* hs, HostPool* pool, bool single = false)
      : t_(t), h_sym_(h_sym), h_sym16_(h_sym16), h_idx8_(h_idx8), hs_(hs), pool_(pool), B_(B) {
    dec_.resize(single ? 1 : B);
    for (size_t b = 0; b < dec_.size(); ++b) dec_[b].set_stream(y[b], ylen[b]);
  }
  // one phase: uint8 indexes D2H, host rANS decode, symbols H2D as int16 -- or as int32 when one of
  // the phase's symbols does not fit (returns false: cb->sym then holds them, not cb->sym16)
  bool run(int64_t n_per, hipStream_t st, const CoderBufs& cb) {
    const int B = B_;
    HIP_OK(hipMemcpyAsync(h_idx8_, cb.idx8, (size_t)n_per * B, hipMemcpyDeviceToHost, st));
    {
      HostStats::Scope w{hs_->wait_ns};
      HIP_OK(hipStreamSynchronize(st));
    }
    const int parts = ((int)dec_.size() == 1 && B > 1) ? 1 : B;  // one batched stream: [B][n_per] in order
    const int64_t n = parts == 1 ? n_per * B : n_per;
    std::vector<char> wide(parts, 0);
    auto work = [&](int b) {
      HostStats::Scope d{hs_->dec_ns};
      if (!rans_decode_piece(dec_[b], h_idx8_ + b * n, n, *t_, h_sym16_ + b * n, h_sym_ + b * n)) wide[b] = 1;
    };
    if (parts == 1) work(0);
    else pool_->run(B, work, HostPool::DECODE);
    bool narrow = true;
    for (char w : wide) narrow = narrow && !w;
    if (!narrow) {  // widen the parts that fit int16 beside the ones decoded as int32
      for (int b = 0; b < parts; ++b)
        if (!wide[b])
          for (int64_t i = 0; i < n; ++i) h_sym_[b * n + i] = h_sym16_[b * n + i];
      HIP_OK(hipMemcpyAsync(cb.sym, h_sym_, sizeof(int32_t) * n_per * B, hipMemcpyHostToDevice, st));
    } else {
      HIP_OK(hipMemcpyAsync(cb.sym16, h_sym16_, sizeof(int16_t) * n_per * B, hipMemcpyHostToDevice, st));
    }
    return narrow;
  }

 private:
  std::vector<RansDecoderState> dec_;
  const CdfTables* t_;
  int32_t* h_sym_;
  int16_t* h_sym16_;
  uint8_t* h_idx8_;
  HostStats* hs_;
  HostPool* pool_;
  int B_;
};

// mlicpp.py:107-176 (forward), 220-277 (compress), 309-366 (decompress)
void Model::slice_loop(Mode mode, const View& hyper, const View* y, const View& yhat, float* y_lik, const CoderBufs* cb,
                       PhaseDecoder* dec) {
  const int S = cfg_.S, C = cfg_.C, hM = cfg_.hM();
  const int H = hyper.H, W = hyper.W, HW = H * W;
  const int64_t n_per = (int64_t)C * H * (W / 2);
  const View hyper_means = hyper.ch(hM, hM);
  View hoisted;  // W_hyp . hyper of all 2 S EntropyParameters (one GEMM, before the serial loop)
  const View* hp = nullptr;
  if (hoist_on() && HW % 4 == 0) {
    hoisted = alloc(hoist_.Cout, H, W);
    conv({hyper}, hoist_, 1, 0, hoisted, EPI_NONE);
    hp = &hoisted;
  }
  float* vbr_dev = nullptr;  // per-image VBR gains [2][B] (gain, 1 / gain)
  if (L().vbr_on) {
    MLIC_CHECK((int)L().vbr_host.size() == 2 * L().B, "vbr scales");
    vbr_dev = L().arena.alloc(2 * L().B);
    if (!L().dry)
      HIP_OK(hipMemcpyAsync(vbr_dev, L().vbr_host.data(), sizeof(float) * 2 * L().B, hipMemcpyHostToDevice, L().st));
  }
  for (int idx = 0; idx < S; ++idx) {
    const size_t m = L().arena.mark();
    View ysl = yhat.ch(idx * C, C);
    View inter, chan, pa;
    if (idx == 0) {
      pa = entropy_parameters({}, &hyper, "anchor", 0, hp, true);
    } else {
      View prev = yhat.ch(0, idx * C);
      inter = inter_context(prev, idx);
      chan = channel_context(prev, idx);
      pa = entropy_parameters({inter, chan}, &hyper, "anchor", idx, hp, true);
    }
    for (int ph = 0; ph < 2; ++ph) {
      QuantParams Q{};
      Q.C = C;
      Q.H = H;
      Q.W = W;
      Q.B = L().B;
      Q.yh = ysl.p;
      Q.yh_bs = ysl.bs;
      Q.table = scale_table_;
      Q.ntable = 64;
      Q.vbr = L().vbr_on ? 1 : 0;
      Q.sc = vbr_dev;
      Q.rs = vbr_dev + L().B;
      Q.phase = ph;
      View pn;
      if (ph == 1) {
        View local = local_context(ysl, idx, ep_half_chain("nonanchor", idx, H, W, hp != nullptr));
        if (idx == 0) {
          pn = entropy_parameters({local}, &hyper, "nonanchor", 0, hp, true);
        } else {
          View intra = intra_context(yhat.ch((idx - 1) * C, C), ysl, idx);
          pn = entropy_parameters({local, intra, inter, chan}, &hyper, "nonanchor", idx, hp, true);
        }
      }
      const View& par = ph == 0 ? pa : pn;
      Q.params = par.p;
      Q.params_bs = par.bs;
      const int phase_id = 2 * idx + ph;
      if (mode == Mode::Decode) {
        Q.idx8 = cb->idx8;
        Q.sym = cb->sym;
        if (!L().dry) {
          phase_indexes(Q, L().st);
          Q.sym16 = dec->run(n_per, L().st, *cb) ? cb->sym16 : nullptr;
          phase_dequant(Q, L().st);
        }
      } else {
        Q.y = y->p + (int64_t)idx * C * HW;
        Q.y_bs = y->bs;
        if (ph == 1 && mode != Mode::Decode && y_lik) {
          Q.lik = y_lik + (int64_t)idx * C * HW;
          Q.lik_bs = (int64_t)cfg_.M * HW;
          Q.params_a = pa.p;
          Q.params_a_bs = pa.bs;
        }
        if (mode == Mode::Encode) {
          const int64_t off = (int64_t)phase_id * L().B * n_per;
          Q.sym = cb->sym + off;
          Q.sym16 = cb->sym16 + off;
          Q.idx8 = cb->idx8 + off;
          Q.ovf = cb->ovf;
          Q.nlim = narrow_limit();
        }
        timed(PCAT_ELEM, 0.0, 4.0 * L().B * C * HW * 5, [&] { quant_phase(Q, L().st); }, "quant_phase");
        Lane& l = L();
        if (mode == Mode::Encode && l.phase_d2h && !l.dry && phase_d2h_mode() != 0) {
          // this phase's coder inputs leave now: on the lane's copy stream (mode 1), or in the lane's
          // own stream order (mode 2: no extra stream -- streams beyond the box's hardware queues
          // share them, and a queued wait would hold another lane's kernels)
          const int64_t off = (int64_t)phase_id * l.B * n_per, nb = l.B * n_per;
          hipStream_t cs = l.st;
          if (phase_d2h_mode() == 1) {
            HIP_OK(hipEventRecord(l.cev, l.st));
            HIP_OK(hipStreamWaitEvent(l.cst, l.cev, 0));
            cs = l.cst;
          }
          HIP_OK(hipMemcpyAsync(l.hc_sym16 + off, Q.sym16, sizeof(int16_t) * nb, hipMemcpyDeviceToHost, cs));
          HIP_OK(hipMemcpyAsync(l.hc_idx8 + off, Q.idx8, nb, hipMemcpyDeviceToHost, cs));
        }
      }
      // LRP on cat([hyper_means] + y_hat_slices + [current])
      // compress: the last slice's final y_hat feeds nothing (no later slice; compress() decodes nothing),
      // so its non-anchor LRP is skipped (mlicpp.py:275-276 computes and discards it)
      if (mode == Mode::Encode && idx == S - 1 && ph == 1) continue;
      lrp({hyper_means, yhat.ch(0, (idx + 1) * C)}, ph == 0 ? "anchor" : "nonanchor", idx, ysl, ph == 0);
    }
    L().arena.release(m);
  }
}

void Model::eb(const View& z, const View& z_hat, float* z_lik, int32_t* z_sym) {
  EbParams P{};
  const std::string p = "entropy_bottleneck";
  P.z = z.p;
  P.z_hat = z_hat.p;
  P.lik = z_lik;
  P.sym = z_sym;
  P.quantiles = rw(p + ".quantiles");
  P.m0 = rw(p + "._matrix0"); P.m1 = rw(p + "._matrix1"); P.m2 = rw(p + "._matrix2");
  P.m3 = rw(p + "._matrix3"); P.m4 = rw(p + "._matrix4");
  P.b0 = rw(p + "._bias0"); P.b1 = rw(p + "._bias1"); P.b2 = rw(p + "._bias2");
  P.b3 = rw(p + "._bias3"); P.b4 = rw(p + "._bias4");
  P.f0 = rw(p + "._factor0"); P.f1 = rw(p + "._factor1"); P.f2 = rw(p + "._factor2"); P.f3 = rw(p + "._factor3");
  P.C = z.C;
  P.H = z.H;
  P.W = z.W;
  P.B = L().B;
  timed(PCAT_ELEM, 0.0, 12.0 * L().B * z.C * z.H * z.W, [&] { eb_forward(P, L().st); }, "entropy_bottleneck");
}

template <class F>
void Model::planned(int B, hipStream_t st, F&& body) {
  Lane& l = L();
  l.B = B;
  (void)st;  // the stream is chosen by the caller of planned() (lane's own or the API caller's)
  l.dry = true;
  l.arena.begin(true);
  body();
  const size_t need = l.arena.peak();
  l.dry = false;
  l.arena.ensure(need + (1 << 20));
  l.arena.begin(false);
  if (poison_) l.arena.poison_on(l.st);
  struct Off {
    Arena& a;
    ~Off() { a.poison_off(); }
  } off{l.arena};
  body();
}

void Model::ensure_host(size_t n) {
  Lane& l = L();
  if (n <= l.h_cap) return;
  for (void* p : {(void*)l.h_sym, (void*)l.h_sym16, (void*)l.h_idx8})
    if (p) HIP_OK(hipHostFree(p));
  l.h_sym = nullptr;
  l.h_sym16 = nullptr;
  l.h_idx8 = nullptr;
  HIP_OK(hipHostMalloc(&l.h_sym, n * sizeof(int32_t)));
  HIP_OK(hipHostMalloc(&l.h_sym16, n * sizeof(int16_t)));
  HIP_OK(hipHostMalloc(&l.h_idx8, n));
  l.h_cap = n;
}

// where compress's per-phase coder inputs go to the host: $MLIC_PHASE_D2H = 0 (default) one copy of all
// phases after the network, 1 each phase on the lane's copy stream as soon as it is quantised, 2 each
// phase in the lane's own stream order.  Measured (alternating pairs, one box): main 87.7 img/s with
// mode 0 against 84.5 with mode 1, Kodak-size 391 against 381 -- the copies run as blit kernels
// (__amd_rocclr_copyBuffer) on the CUs, and 20 of them per call beside the network cost more than the
// one copy they save at the end; an extra stream per lane also shares the box's 4 hardware queues
int Model::phase_d2h_mode() {
  static const int m = [] {
    const char* e = std::getenv("MLIC_PHASE_D2H");
    return e ? std::atoi(e) : 0;
  }();
  return m;
}

void Model::ensure_chost(size_t n) {
  Lane& l = L();
  if (!l.cst && phase_d2h_mode() == 1) {  // (no extra stream unless it is used)
    HIP_OK(hipStreamCreateWithFlags(&l.cst, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&l.cev, hipEventDisableTiming));
  }
  if (n <= l.hc_cap) return;
  for (void* p : {(void*)l.hc_sym, (void*)l.hc_sym16, (void*)l.hc_idx8})
    if (p) HIP_OK(hipHostFree(p));
  l.hc_sym = nullptr;
  l.hc_sym16 = nullptr;
  l.hc_idx8 = nullptr;
  HIP_OK(hipHostMalloc(&l.hc_sym, n * sizeof(int32_t)));
  HIP_OK(hipHostMalloc(&l.hc_sym16, n * sizeof(int16_t)));
  HIP_OK(hipHostMalloc(&l.hc_idx8, n));
  l.hc_cap = n;
}

void Model::set_vbr(const float* scales, int B) {
  Lane& l = L();
  l.vbr_on = cfg_.vbr;
  l.vbr_host.assign(2 * B, 1.0f);
  if (!l.vbr_on) return;
  for (int b = 0; b < B; ++b) {
    const float s = scales ? scales[b] : 1.0f;
    // forward uses Gain[s] as stored (mlicpp_vbr.py:122-135); compress/decompress receive |Gain[s]|
    // from the Python layer (mlicpp_vbr.py:543, 899)
    MLIC_CHECK(std::isfinite(s) && s != 0.0f, "VBR gain must be finite and nonzero");
    l.vbr_host[b] = s;
    l.vbr_host[B + b] = 1.0f / s;  // mlicpp_vbr.py: rescale by 1 / scale
  }
}

hipEvent_t Model::next_event() {
  Lane& l = L();
  if (l.ev_used == l.ev_pool.size()) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    l.ev_pool.push_back(e);
  }
  return l.ev_pool[l.ev_used++];
}

template <class F>
void Model::timed(int cat, double flops, double bytes, F&& launch, const std::string& tag) {
  Lane& l = L();
  if (l.dry) return;
  if (!l.prof) {
    launch();
    return;
  }
  Lane::ProfRec r;
  r.a = next_event();
  r.b = next_event();
  r.cat = cat;
  r.flops = flops;
  r.bytes = bytes;
  r.tag = tag;
  HIP_OK(hipEventRecord(r.a, l.st));
  launch();
  HIP_OK(hipEventRecord(r.b, l.st));
  l.recs.push_back(r);
}

std::string Model::profile_layers() {
  struct Acc {
    int64_t n = 0;
    double ms = 0, flops = 0, bytes = 0;
    int cat = 0;
  };
  std::map<std::string, Acc> acc;
  for (auto& lp : lanes_)
    for (auto& r : lp->recs) {
      if (r.tag.empty()) continue;
      // group per-slice layers: drop the digits after the first dot-separated component index
      HIP_OK(hipEventSynchronize(r.b));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, r.a, r.b));
      Acc& a = acc[r.tag];
      a.n++;
      a.ms += ms;
      a.flops += r.flops;
      a.bytes += r.bytes;
      a.cat = r.cat;
    }
  std::vector<std::pair<std::string, Acc>> v(acc.begin(), acc.end());
  std::sort(v.begin(), v.end(), [](auto& x, auto& y) { return x.second.ms > y.second.ms; });
  std::string out = "layer\tkernel\tlaunches\tms\tGFLOP\tTFLOP/s\tGB\tGB/s\n";
  char buf[512];
  for (auto& kv : v) {
    const Acc& a = kv.second;
    std::snprintf(buf, sizeof buf, "%s\t%s\t%lld\t%.4f\t%.3f\t%.2f\t%.3f\t%.0f\n", kv.first.c_str(),
                  prof_cat_name(a.cat), (long long)a.n, a.ms, a.flops / 1e9,
                  a.ms > 0 ? a.flops / (a.ms * 1e-3) / 1e12 : 0.0, a.bytes / 1e9,
                  a.ms > 0 ? a.bytes / (a.ms * 1e-3) / 1e9 : 0.0);
    out += buf;
  }
  return out;
}

ProfStat Model::profile_read(int cat) {
  ProfStat s;
  for (auto& lp : lanes_) {
    Lane& l = *lp;
    std::vector<Lane::ProfRec> keep;
    for (auto& r : l.recs) {
      if (r.cat != cat) {
        keep.push_back(r);
        continue;
      }
      HIP_OK(hipEventSynchronize(r.b));
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, r.a, r.b));
      s.launches += 1;
      s.ms += ms;
      s.flops += r.flops;
      s.bytes += r.bytes;
    }
    l.recs.swap(keep);
    if (l.recs.empty()) l.ev_used = 0;
  }
  return s;
}

template <class F>
void Model::over_lanes(int B, hipStream_t caller, F&& fn, int max_lanes) {
  const int nl = std::max(1, std::min(std::min(nlanes_, max_lanes), B));
  hipEvent_t ready;
  HIP_OK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  HIP_OK(hipEventRecord(ready, caller));  // inputs produced on the caller's stream
  std::vector<std::exception_ptr> errs(nl);
  std::vector<std::thread> th;
  int first = 0;
  for (int i = 0; i < nl; ++i) {
    const int cnt = B / nl + (i < B % nl ? 1 : 0);
    Lane& l = lane(i);
    HIP_OK(hipStreamWaitEvent(l.st, ready, 0));
    th.emplace_back([&, i, first, cnt, &l = l] {
      tl_lane_ = &l;
      try {
        fn(l, first, cnt);
      } catch (...) {
        errs[i] = std::current_exception();
      }
      tl_lane_ = nullptr;
    });
    first += cnt;
  }
  for (auto& t : th) t.join();
  for (int i = 0; i < nl; ++i) {  // outputs visible to the caller's stream
    hipEvent_t done;
    HIP_OK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    HIP_OK(hipEventRecord(done, lanes_[i]->st));
    HIP_OK(hipStreamWaitEvent(caller, done, 0));
    HIP_OK(hipEventDestroy(done));
  }
  HIP_OK(hipEventDestroy(ready));
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// ------------------------------------------------------------------------------------- entry points
void Model::forward(const float* x, int B, int H, int W, float* x_hat, float* y_lik, float* z_lik, const float* vbr_scales,
                    hipStream_t st) {
  MLIC_CHECK(H % 64 == 0 && W % 64 == 0, "H and W must be multiples of 64 (pad like utils/testing.py:130-137)");
  // forward() runs on the caller's stream in lane 0 (torch-ordered)
  Lane& l = lane(0);
  hipStream_t own = l.st;
  tl_lane_ = &l;
  struct Restore {
    Lane& l;
    hipStream_t s;
    ~Restore() { l.st = s; l.prec_force = -1; tl_lane_ = nullptr; }
  } restore{l, own};
  l.st = st;  // caller's stream, including the legacy NULL stream torch uses by default
  set_vbr(vbr_scales, B);
  range_clear(l);
  // The fp16 range guard needs a device-to-host read, i.e. a synchronisation of `st`; under stream
  // capture (hipGraph) there is none, and a captured forward cannot fall back: its flag stays set
  // for the caller to read.  Otherwise forward() returns with `st` synchronised.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_OK(hipStreamIsCapturing(st, &cap));
  const bool guard = cap == hipStreamCaptureStatusNone && prec() != PREC_F32;
  bool entropy_hit = false;
  View yhat;
  const View out{x_hat, 3, H, W, (int64_t)3 * H * W};
  auto body = [&] {
    View xv{const_cast<float*>(x), 3, H, W, (int64_t)3 * H * W};
    View y = g_a(xv);
    View z = h_a(y);
    View zh = alloc(z.C, z.H, z.W);
    eb(z, zh, z_lik, nullptr);
    View hyper = h_s(zh);
    yhat = alloc(cfg_.M, y.H, y.W);
    slice_loop(Mode::Forward, hyper, &y, yhat, y_lik, nullptr, nullptr);
    // the same policy as compress / decompress: an overflow in the entropy model (g_a .. slice loop)
    // re-runs the whole call in exact fp32 (compress refuses such an input); one in g_s alone re-runs
    // g_s alone, as decompress does, so decompress(compress(x)) == forward(x) bit for bit
    if (guard && !l.dry && prec() != PREC_F32) entropy_hit = range_hit(l);
    if (x_hat && !entropy_hit) g_s(yhat, out);
  };
  planned(B, st, body);
  if (entropy_hit) {
    fb_.forward_full++;
    entropy_hit = false;
    l.prec_force = PREC_F32;
    planned(B, st, body);
    l.prec_force = -1;
    (void)range_hit(l);
    return;
  }
  if (guard && range_hit(l) && x_hat) {
    fb_.forward_gs++;
    gs_fp32_rerun(l, yhat, out, B);
  }
}

void Model::gs_fp32_rerun(Lane& l, const View& yhat, const View& out, int B) {
  const size_t nb = sizeof(float) * (size_t)B * yhat.bs;
  float* keep = nullptr;
  HIP_OK(hipMalloc(&keep, nb));
  struct Free {
    float* p;
    Lane& l;
    ~Free() { l.prec_force = -1; (void)hipStreamSynchronize(l.st); (void)hipFree(p); }
  } fr{keep, l};
  HIP_OK(hipMemcpyAsync(keep, yhat.p, nb, hipMemcpyDeviceToDevice, l.st));
  l.prec_force = PREC_F32;
  planned(B, l.st, [&] { g_s(View{keep, yhat.C, yhat.H, yhat.W, yhat.bs}, out); });
  l.prec_force = -1;
  (void)range_hit(l);
}

// the fp16 range guard (common.h range_check): read and clear the lane's device flag
bool Model::range_hit(Lane& l) {
  int h = 0;
  HIP_OK(hipMemcpyAsync(&h, l.rflag, sizeof(int), hipMemcpyDeviceToHost, l.st));
  HIP_OK(hipStreamSynchronize(l.st));
  if (h) HIP_OK(hipMemsetAsync(l.rflag, 0, sizeof(int), l.st));
  return h != 0;
}

void Model::range_clear(Lane& l) { HIP_OK(hipMemsetAsync(l.rflag, 0, sizeof(int), l.st)); }

// compress/decompress cannot fall back silently for the entropy model: the decoder has to reproduce
// the encoder's exact entropy parameters, so both sides must run the same arithmetic
static const char* kRangeMsg =
    "mlic: an activation of the entropy model exceeded the fp16 range of the split-fp16 kernels (|v| >= 65504); "
    "encode and decode this input with set_precision(0) (exact fp32 MFMA)";

void Model::compress(const float* x, int B, int H, int W, const float* vbr_scales, hipStream_t st) {
  MLIC_CHECK(H % 64 == 0 && W % 64 == 0, "H and W must be multiples of 64");
  MLIC_CHECK(!gc_.empty() && !eb_.empty(), "entropy tables not set: call update() first");
  enc_all_.assign(B, EncodedImage{});
  const int64_t img = (int64_t)3 * H * W;
  over_lanes(B, st, [&](Lane& l, int first, int cnt) {
    set_vbr(vbr_scales ? vbr_scales + first : nullptr, cnt);
    compress_lane(x + first * img, cnt, H, W);
    for (int b = 0; b < cnt; ++b) enc_all_[first + b] = std::move(l.enc[b]);
  });
}

// mlicpp.py:199-290 for the lane's images: network on the lane stream, then one host thread per
// image runs the rANS coder over that image's 20 phase streams (+ the z stream)
void Model::compress_lane(const float* x, int B, int H, int W) {
  Lane& l = L();
  const int h = H / 16, w = W / 16, hz = H / 64, wz = W / 64;
  const int64_t n_per = (int64_t)cfg_.C * h * (w / 2);
  const int nph = 2 * cfg_.S;
  const int64_t ny = (int64_t)nph * B * n_per, nz = (int64_t)B * cfg_.N * hz * wz;
  int32_t* d_zsym = nullptr;
  CoderBufs cb;
  double* d_bits = nullptr;  // [2][B]: -log2 likelihood sums of y and z per image (B1, rd_loss.py:42-45)
  range_clear(l);
  ensure_chost((size_t)(ny + nz));
  l.phase_d2h = true;
  struct Off {
    Lane& l;
    ~Off() { l.phase_d2h = false; }
  } phase_off{l};
  planned(B, nullptr, [&] {
    cb.sym = reinterpret_cast<int32_t*>(l.arena.alloc(ny));
    cb.sym16 = reinterpret_cast<int16_t*>(l.arena.alloc((ny + 1) / 2));
    cb.idx8 = reinterpret_cast<uint8_t*>(l.arena.alloc((ny + 3) / 4));
    cb.ovf = reinterpret_cast<int*>(l.arena.alloc(1));
    if (!l.dry) HIP_OK(hipMemsetAsync(cb.ovf, 0, sizeof(int), l.st));
    d_zsym = reinterpret_cast<int32_t*>(l.arena.alloc(nz));
    d_bits = reinterpret_cast<double*>(l.arena.alloc(4 * B));
    double* part = reinterpret_cast<double*>(l.arena.alloc(4 * neglog2_partial_doubles(B)));
    const int64_t ny_img = (int64_t)cfg_.M * h * w, nz_img = (int64_t)cfg_.N * hz * wz;
    float* y_lik = l.arena.alloc(B * ny_img);
    float* z_lik = l.arena.alloc(B * nz_img);
    View xv{const_cast<float*>(x), 3, H, W, (int64_t)3 * H * W};
    View y = g_a(xv);
    View z = h_a(y);
    View zh = alloc(z.C, z.H, z.W);
    eb(z, zh, z_lik, d_zsym);  // z_hat = round(z - med) + med == decompress(compress(z))
    View hyper = h_s(zh);
    View yhat = alloc(cfg_.M, y.H, y.W);
    slice_loop(Mode::Encode, hyper, &y, yhat, y_lik, &cb, nullptr);
    timed(PCAT_ELEM, 0.0, 4.0 * B * (ny_img + nz_img), [&] {
      neglog2_sum(y_lik, ny_img, B, d_bits, part, l.st);
      neglog2_sum(z_lik, nz_img, B, d_bits + B, part + neglog2_partial_doubles(B), l.st);
    }, "bpp_lik");
  });
  std::vector<double> bits(2 * B);
  HIP_OK(hipMemcpyAsync(bits.data(), d_bits, sizeof(double) * 2 * B, hipMemcpyDeviceToHost, l.st));
  int32_t* hzs = l.hc_sym + ny;
  // the coder inputs cross PCIe narrow: int16 symbols + uint8 scale indexes (3 B instead of 8 per
  // symbol); a symbol beyond int16 (set *ovf) brings the int32 copy instead
  int ovf = 0;
  if (phase_d2h_mode() == 0) {  // every phase in one copy after the network
    HIP_OK(hipMemcpyAsync(l.hc_sym16, cb.sym16, ny * sizeof(int16_t), hipMemcpyDeviceToHost, l.st));
    HIP_OK(hipMemcpyAsync(l.hc_idx8, cb.idx8, ny, hipMemcpyDeviceToHost, l.st));
  }
  HIP_OK(hipMemcpyAsync(hzs, d_zsym, nz * 4, hipMemcpyDeviceToHost, l.st));
  HIP_OK(hipMemcpyAsync(&ovf, cb.ovf, sizeof(int), hipMemcpyDeviceToHost, l.st));
  {
    HostStats::Scope w{hstats_.wait_ns};
    HIP_OK(hipStreamSynchronize(l.st));
    if (phase_d2h_mode() == 1) HIP_OK(hipStreamSynchronize(l.cst));
    if (ovf) {
      HIP_OK(hipMemcpyAsync(l.hc_sym, cb.sym, ny * 4, hipMemcpyDeviceToHost, l.st));
      HIP_OK(hipStreamSynchronize(l.st));
    }
  }
  if (prec() != PREC_F32 && range_hit(l)) throw Error(kRangeMsg);
  l.enc.assign(B, EncodedImage{});
  for (int b = 0; b < B; ++b) {
    l.enc[b].y_bits = bits[b];
    l.enc[b].z_bits = bits[B + b];
  }
  const int64_t zper = (int64_t)cfg_.N * hz * wz;
  auto work = [&](int b) {
    HostStats::Scope e{hstats_.enc_ns};
    // y: phases in order, this image's part of each ([phase][B][n_per] in the pinned buffers), coded
    // straight from there: rANS codes LIFO, so the last phase goes in first
    CoderView v{ovf ? l.hc_sym + b * n_per : nullptr, ovf ? nullptr : l.hc_sym16 + b * n_per, l.hc_idx8 + b * n_per,
                n_per, (int64_t)B * n_per, nph};
    RansEncoder enc(v.size());
    for (int k = nph; k-- > 0;) v.put_phase(enc, k, gc_);
    l.enc[b].y = enc.flush();
    l.enc[b].y_in = v;
    l.enc[b].z_sym.assign(hzs + b * zper, hzs + (b + 1) * zper);
    // z: EntropyBottleneck._build_indexes -> channel index, C-order over [C, hz, wz]
    std::vector<int32_t> zi(zper);
    for (int64_t i = 0; i < zper; ++i) zi[i] = (int32_t)(i / ((int64_t)hz * wz));
    l.enc[b].z = rans_encode(hzs + b * zper, zi.data(), zper, eb_);
  };
  host_pool().run(B, work);
}

// one process-wide pool (every handle's lanes submit to it): a sweep over several weight sets does
// not multiply the coder threads; $MLIC_HOST_THREADS (bench.py sets cores / ranks-per-node)
HostPool& Model::host_pool() {
  static std::once_flag once;
  static std::unique_ptr<HostPool> pool;
  std::call_once(once, [] {
    int n = (int)std::thread::hardware_concurrency();
    if (const char* e = std::getenv("MLIC_HOST_THREADS")) n = std::atoi(e);
    n = std::max(1, std::min(n, 16));
    pool = std::make_unique<HostPool>(n);
  });
  return *pool;
}

void Model::decompress(const uint8_t* const* y, const size_t* ylen, const uint8_t* const* z, const size_t* zlen,
                       int B, int hz, int wz, float* x_hat, const float* vbr_scales, hipStream_t st, bool batch_stream) {
  MLIC_CHECK(!gc_.empty() && !eb_.empty(), "entropy tables not set: call update() first");
  const int64_t img = (int64_t)3 * 64 * hz * 64 * wz;
  over_lanes(B, st, [&](Lane& l, int first, int cnt) {
    set_vbr(vbr_scales ? vbr_scales + first : nullptr, cnt);
    decompress_lane(batch_stream ? y : y + first, batch_stream ? ylen : ylen + first, z + first, zlen + first, cnt, hz,
                    wz, x_hat + first * img, batch_stream);
  }, batch_stream ? 1 : 16);
}

std::string Model::batch_stream(int first, int count) const {
  MLIC_CHECK(first >= 0 && count >= 1 && first + count <= (int)enc_all_.size(), "batch_stream: image range");
  const CoderView& v0 = enc_all_[first].y_in;
  const int64_t n_per = v0.n_per;
  for (int b = first; b < first + count; ++b)
    MLIC_CHECK(enc_all_[b].y_in.n_per == n_per && enc_all_[b].y_in.nph == v0.nph, "batch_stream: images of one shape");
  // phase-major, image-minor: coded LIFO, so the last phase's last image goes in first
  RansEncoder enc(v0.size() * count);
  for (int k = v0.nph; k-- > 0;)
    for (int b = first + count; b-- > first;) {
      enc_all_[b].y_in.put_phase(enc, k, gc_);
    }
  return enc.flush();
}

// mlicpp.py:292-378 for the lane's images: z decoded on the host, then 20 phases of
// (network -> indexes D2H -> per-image host rANS decode -> symbols H2D -> dequantise)
void Model::decompress_lane(const uint8_t* const* y, const size_t* ylen, const uint8_t* const* z,
                            const size_t* zlen, int B, int hz, int wz, float* x_hat, bool batch_stream) {
  Lane& l = L();
  const int h = hz * 4, w = wz * 4;
  const int64_t n_per = (int64_t)cfg_.C * h * (w / 2);
  const int64_t zper = (int64_t)cfg_.N * hz * wz;
  ensure_host((size_t)std::max<int64_t>(B * n_per, B * zper));
  {
    std::vector<int32_t> zi(zper);
    for (int64_t i = 0; i < zper; ++i) zi[i] = (int32_t)(i / ((int64_t)hz * wz));
    host_pool().run(B, [&](int b) {  // one z stream per image, decoded in parallel
      HostStats::Scope d{hstats_.dec_ns};
      RansDecoderState dz;
      dz.set_stream(z[b], zlen[b]);
      dz.decode(zi.data(), zper, eb_, l.h_sym + b * zper);
    }, HostPool::DECODE);
  }
  PhaseDecoder dec(B, y, ylen, &gc_, l.h_sym, l.h_sym16, l.h_idx8, &hstats_, &host_pool(), batch_stream);
  const int32_t* hz_sym = l.h_sym;
  range_clear(l);
  View yhat;
  const View out{x_hat, 3, 16 * h, 16 * w, (int64_t)3 * 16 * h * 16 * w};
  planned(B, nullptr, [&] {
    int32_t* d_zsym = reinterpret_cast<int32_t*>(l.arena.alloc(B * zper));
    CoderBufs cb;
    cb.sym = reinterpret_cast<int32_t*>(l.arena.alloc(B * n_per));
    cb.sym16 = reinterpret_cast<int16_t*>(l.arena.alloc((B * n_per + 1) / 2));
    cb.idx8 = reinterpret_cast<uint8_t*>(l.arena.alloc((B * n_per + 3) / 4));
    View zh = alloc(cfg_.N, hz, wz);
    if (!l.dry) {
      HIP_OK(hipMemcpyAsync(d_zsym, hz_sym, B * zper * 4, hipMemcpyHostToDevice, l.st));
      eb_dequant(d_zsym, rw("entropy_bottleneck.quantiles"), zh.p, cfg_.N, hz * wz, B, l.st);
      HIP_OK(hipStreamSynchronize(l.st));  // the z symbols' host buffer is reused by the phase decoder
    }
    View hyper = h_s(zh);
    yhat = alloc(cfg_.M, h, w);
    slice_loop(Mode::Decode, hyper, nullptr, yhat, nullptr, &cb, &dec);
    // the entropy model (h_s + slice loop) must match the encoder's arithmetic: no fallback there
    if (!l.dry && prec() != PREC_F32 && range_hit(l)) throw Error(kRangeMsg);
    g_s(yhat, out);
  });
  if (prec() != PREC_F32 && range_hit(l)) {
    // only the synthesis transform left fp16's range: y_hat is final, so re-run g_s alone in exact
    // fp32 MFMA (forward() takes the same fallback)
    fb_.decompress_gs++;
    gs_fp32_rerun(l, yhat, out, B);
  }
}

// module-level entry points (tests): which in {local, chan, inter, intra, epa, epn, lrpa, lrpn, g_a, h_a, h_s, g_s, rbu}
void Model::run_module(const std::string& which, int i, const float* in0, const float* in1, int B, int Cin, int H,
                       int W, float* out, hipStream_t st) {
  Lane& l = lane(0);
  hipStream_t own = l.st;
  tl_lane_ = &l;
  struct Restore {
    Lane& l;
    hipStream_t s;
    ~Restore() { l.st = s; tl_lane_ = nullptr; }
  } restore{l, own};
  l.st = st;
  range_clear(l);  // a stale hit of an earlier call must not be reported against this one
  planned(B, st, [&] {
    View a{const_cast<float*>(in0), Cin, H, W, (int64_t)Cin * H * W};
    View r;
    if (which == "local") r = local_context(a, i);
    else if (which == "chan") r = channel_context(a, i);
    else if (which == "inter") r = inter_context(a, i);
    else if (which == "intra") {
      View b{const_cast<float*>(in1), Cin, H, W, (int64_t)Cin * H * W};
      r = intra_context(a, b, i);
    } else if (which == "epa") r = entropy_parameters({a}, nullptr, "anchor", i);
    else if (which == "epn") r = entropy_parameters({a}, nullptr, "nonanchor", i);
    else if (which == "g_a") r = g_a(a);
    else if (which == "h_a") r = h_a(a);
    else if (which == "h_s") r = h_s(a);
    else if (which == "rbu") r = rbu(a, "g_s.synthesis_transform." + std::to_string(i));
    else if (which == "rbws") r = rbws(a, "g_a.analysis_transform." + std::to_string(i), !cfg_.sd);
    else if (which == "g_s") {
      View o{out, 3, 16 * H, 16 * W, (int64_t)3 * 256 * H * W};
      g_s(a, o);
      return;
    } else if (which == "lrpn") {
      // in0 = LRP input, in1 = residual slice (copied to out first); out = res + mask(0.5 tanh(lrp(x)))
      View o{out, cfg_.C, H, W, (int64_t)cfg_.C * H * W};
      if (!L().dry) HIP_OK(hipMemcpyAsync(out, in1, sizeof(float) * B * o.bs, hipMemcpyDeviceToDevice, L().st));
      lrp({a}, "nonanchor", i, o, false);
      return;
    } else throw Error("mlic: unknown module " + which);
    if (!L().dry) HIP_OK(hipMemcpyAsync(out, r.p, sizeof(float) * B * r.bs, hipMemcpyDeviceToDevice, L().st));
  });
}

}  // namespace mlic
