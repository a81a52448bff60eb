// Host rANS coder, byte-compatible with compressai 1.2.6 (cpp_exts/rans/rans_interface.cpp on top
// of ryg_rans' rans64.h): 64-bit state, RANS64_L = 2^31, 32-bit output words (little endian),
// 16-bit CDF precision, out-of-range values escaped with 4-bit "bypass" symbols.  Restated from
// the published algorithm; the reference calls it at models/mlicpp.py:215,279-281,306-307 and
// utils/ckbd.py:199,217.  Symbols are pushed in call order and coded LIFO at flush, so the
// decoder reads them back in call order.
#include "rans.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <stdexcept>

namespace mlic {

namespace {
constexpr uint64_t RANS64_L = 1ull << 31;
constexpr int PRECISION = 16;
constexpr int BYPASS_PRECISION = 4;
constexpr int MAX_BYPASS_VAL = (1 << BYPASS_PRECISION) - 1;

struct Sym {
  uint16_t start;
  uint16_t range;
  bool bypass;
};

inline void enc_put(uint64_t& x, uint32_t*& ptr, uint32_t start, uint32_t freq, uint32_t scale_bits) {
  const uint64_t x_max = ((RANS64_L >> scale_bits) << 32) * freq;
  if (x >= x_max) {
    *--ptr = (uint32_t)x;
    x >>= 32;
  }
  x = ((x / freq) << scale_bits) + (x % freq) + start;
}

inline void enc_put_bits(uint64_t& x, uint32_t*& ptr, uint32_t val, uint32_t nbits) {
  const uint32_t freq = 1u << (16 - nbits);
  const uint64_t x_max = ((RANS64_L >> 16) << 32) * freq;
  if (x >= x_max) {
    *--ptr = (uint32_t)x;
    x >>= 32;
  }
  x = (x << nbits) | val;
}
}  // namespace

std::string rans_encode(const int32_t* symbols, const int32_t* indexes, int64_t n, const CdfTables& t) {
  std::vector<Sym> syms;
  syms.reserve((size_t)n + 16);
  for (int64_t i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    if (ci < 0 || ci >= t.n) throw std::runtime_error("rans: cdf index out of range");
    const int32_t* cdf = t.cdf.data() + (int64_t)ci * t.stride;
    const int32_t max_value = t.length[ci] - 2;
    int32_t value = symbols[i] - t.offset[ci];
    uint32_t raw = 0;
    if (value < 0) {
      raw = (uint32_t)(-2 * value - 1);
      value = max_value;
    } else if (value >= max_value) {
      raw = (uint32_t)(2 * (value - max_value));
      value = max_value;
    }
    syms.push_back({(uint16_t)cdf[value], (uint16_t)(cdf[value + 1] - cdf[value]), false});
    if (value == max_value) {
      int32_t nb = 0;
      while (nb < 8 && (raw >> (nb * BYPASS_PRECISION)) != 0) ++nb;
      int32_t v = nb;
      while (v >= MAX_BYPASS_VAL) {
        syms.push_back({(uint16_t)MAX_BYPASS_VAL, (uint16_t)(MAX_BYPASS_VAL + 1), true});
        v -= MAX_BYPASS_VAL;
      }
      syms.push_back({(uint16_t)v, (uint16_t)(v + 1), true});
      for (int32_t j = 0; j < nb; ++j) {
        const uint32_t bv = (raw >> (j * BYPASS_PRECISION)) & MAX_BYPASS_VAL;
        syms.push_back({(uint16_t)bv, (uint16_t)(bv + 1), true});
      }
    }
  }
  std::vector<uint32_t> out(syms.size() + 4, 0xCCCCCCCCu);
  uint32_t* end = out.data() + out.size();
  uint32_t* ptr = end;
  uint64_t x = RANS64_L;
  for (size_t k = syms.size(); k-- > 0;) {
    const Sym& s = syms[k];
    if (!s.bypass) enc_put(x, ptr, s.start, s.range, PRECISION);
    else enc_put_bits(x, ptr, s.start, BYPASS_PRECISION);
  }
  ptr -= 2;  // flush
  ptr[0] = (uint32_t)(x >> 0);
  ptr[1] = (uint32_t)(x >> 32);
  const size_t nbytes = (size_t)(end - ptr) * sizeof(uint32_t);
  return std::string(reinterpret_cast<const char*>(ptr), nbytes);
}

void RansDecoderState::set_stream(const uint8_t* data, size_t nbytes) {
  words_.assign((nbytes + 3) / 4 + 2, 0u);
  std::memcpy(words_.data(), data, nbytes);
  pos_ = 0;
  state_ = (uint64_t)get_word();
  state_ |= (uint64_t)get_word() << 32;
}

uint32_t RansDecoderState::get_word() {
  // reading past the end of a corrupt stream yields zeros instead of faulting
  return pos_ < words_.size() ? words_[pos_++] : 0u;
}

void RansDecoderState::decode(const int32_t* indexes, int64_t n, const CdfTables& t, int32_t* out) {
  constexpr uint64_t mask = (1ull << PRECISION) - 1;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    if (ci < 0 || ci >= t.n) throw std::runtime_error("rans: cdf index out of range");
    const int32_t* cdf = t.cdf.data() + (int64_t)ci * t.stride;
    const int32_t len = t.length[ci];
    const int32_t max_value = len - 2;
    const uint32_t cum = (uint32_t)(state_ & mask);
    // first entry > cum, minus one (cdf is strictly increasing)
    const int32_t s = (int32_t)(std::upper_bound(cdf, cdf + len, (int32_t)cum) - cdf) - 1;
    if (s < 0 || s > max_value) throw std::runtime_error("rans: corrupt stream");
    const uint32_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
    uint64_t x = freq * (state_ >> PRECISION) + (state_ & mask) - start;
    if (x < RANS64_L) x = (x << 32) | get_word();
    state_ = x;
    int32_t value = s;
    if (value == max_value) {
      auto get_bits = [&](uint32_t nb) {
        uint64_t y = state_;
        const uint32_t v = (uint32_t)(y & ((1u << nb) - 1));
        y >>= nb;
        if (y < RANS64_L) y = (y << 32) | get_word();
        state_ = y;
        return v;
      };
      int32_t v = (int32_t)get_bits(BYPASS_PRECISION);
      int32_t nb = v;
      while (v == MAX_BYPASS_VAL) {
        v = (int32_t)get_bits(BYPASS_PRECISION);
        nb += v;
      }
      if (nb > 8) throw std::runtime_error("rans: corrupt bypass length");
      uint32_t raw = 0;
      for (int32_t j = 0; j < nb; ++j) raw |= get_bits(BYPASS_PRECISION) << (j * BYPASS_PRECISION);
      value = (int32_t)(raw >> 1);
      if (raw & 1) value = -value - 1;
      else value += max_value;
    }
    out[i] = value + t.offset[ci];
  }
}

// compressai cpp_exts/ops/ops.cpp pmf_to_quantized_cdf (restated)
std::vector<uint32_t> pmf_to_quantized_cdf(const float* pmf, int n, int precision) {
  for (int i = 0; i < n; ++i)
    if (!(pmf[i] >= 0.0f) || !std::isfinite(pmf[i])) throw std::runtime_error("invalid pmf");
  std::vector<uint32_t> cdf((size_t)n + 1, 0u);
  for (int i = 0; i < n; ++i) cdf[i + 1] = (uint32_t)std::round(pmf[i] * (float)(1 << precision));
  const uint32_t total = std::accumulate(cdf.begin(), cdf.end(), 0u);
  if (total == 0) throw std::runtime_error("zero pmf");
  for (auto& c : cdf) c = (uint32_t)(((uint64_t)(1u << precision) * c) / total);
  std::partial_sum(cdf.begin(), cdf.end(), cdf.begin());
  cdf.back() = 1u << precision;
  for (int i = 0; i < (int)cdf.size() - 1; ++i) {
    if (cdf[i] == cdf[i + 1]) {
      uint32_t best_freq = ~0u;
      int best_steal = -1;
      for (int j = 0; j < (int)cdf.size() - 1; ++j) {
        const uint32_t freq = cdf[j + 1] - cdf[j];
        if (freq > 1 && freq < best_freq) {
          best_freq = freq;
          best_steal = j;
        }
      }
      if (best_steal < 0) throw std::runtime_error("pmf_to_quantized_cdf: cannot steal");
      if (best_steal < i) {
        for (int j = best_steal + 1; j <= i; ++j) cdf[j]--;
      } else {
        for (int j = i + 1; j <= best_steal; ++j) cdf[j]++;
      }
    }
  }
  return cdf;
}

}  // namespace mlic
