// Host rANS coder, byte-compatible with compressai 1.2.6 (cpp_exts/rans/rans_interface.cpp on top
// of ryg_rans' rans64.h): 64-bit state, RANS64_L = 2^31, 32-bit output words (little endian),
// 16-bit CDF precision, out-of-range values escaped with 4-bit "bypass" symbols.  Restated from
// the published algorithm; the reference calls it at models/mlicpp.py:215,279-281,306-307 and
// utils/ckbd.py:199,217.  Symbols are pushed in call order and coded LIFO at flush, so the
// decoder reads them back in call order.
#include "rans.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>
#include <stdexcept>

namespace mlic {

namespace {
constexpr uint64_t RANS64_L = 1ull << 31;
constexpr int PRECISION = 16;
constexpr int BYPASS_PRECISION = 4;
constexpr int MAX_BYPASS_VAL = (1 << BYPASS_PRECISION) - 1;


inline uint64_t mulhi64(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }

// Rans64EncSymbolInit: x' = (x / freq) * 2^16 + x % freq + start computed as
// x + bias + q * (2^16 - freq), q = mulhi(x, rcp) >> shift == x / freq exactly (ryg_rans proof)
EncSym make_enc_sym(uint32_t start, uint32_t freq) {
  EncSym s;
  s.freq = freq;
  s.cmpl_freq = (1u << PRECISION) - freq;
  if (freq < 2) {
    s.rcp_freq = ~0ull;
    s.rcp_shift = 0;
    s.bias = start + (1u << PRECISION) - 1;
  } else {
    uint32_t shift = 0;
    while (freq > (1u << shift)) shift++;
    uint64_t x0 = freq - 1;
    const uint64_t x1 = 1ull << (shift + 31);
    const uint64_t t1 = x1 / freq;
    x0 += (x1 % freq) << 32;
    const uint64_t t0 = x0 / freq;
    s.rcp_freq = t0 + (t1 << 32);
    s.rcp_shift = shift - 1;
    s.bias = start;
  }
  return s;
}

inline void enc_put_sym(uint64_t& x, uint32_t*& ptr, const EncSym& s) {
  const uint64_t x_max = ((RANS64_L >> PRECISION) << 32) * s.freq;
  if (x >= x_max) {  // rare on low-entropy streams: a predictable branch beats a select on the state's path
    *--ptr = (uint32_t)x;
    x >>= 32;
  }
  const uint64_t q = mulhi64(x, s.rcp_freq) >> s.rcp_shift;
  x = x + s.bias + q * s.cmpl_freq;
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

// n_hint = the symbols to come; the first buffer holds n_hint / 16 words (2 bits per symbol; at the bench's
// 0.1-0.5 bits per symbol a stream never grows, a high-rate one doubles a few times).  Round 6: it was one
// word per symbol, zero-filled: 10.4 MB of memset and first-touch page faults per 1080p image, 41.8 MB per
// 4K image, for a few hundred KB of stream
RansEncoder::RansEncoder(int64_t n_hint) : out_((size_t)std::max<int64_t>(n_hint / 16, 0) + 1024, 0u) {
  end_ = out_.data() + out_.size();
  ptr_ = end_;
}

void RansEncoder::grow() {  // keep the written tail at the end of a larger buffer
  const size_t used = (size_t)(end_ - ptr_);
  std::vector<uint32_t> bigger(out_.size() * 2 + 64, 0u);
  std::memcpy(bigger.data() + bigger.size() - used, ptr_, used * 4);
  out_.swap(bigger);
  end_ = out_.data() + out_.size();
  ptr_ = end_ - used;
}

template <class S, class I>
void RansEncoder::put_reverse(const S* symbols, const I* indexes, int64_t n, const CdfTables& t) {
  if (t.enc.empty()) throw std::runtime_error("rans: tables not prepared");
  // One reverse pass.  compressai pushes, per symbol: the symbol (value clamped to max_value) and,
  // if escaped, the bypass length nb (< 15 for 32-bit values) and nb 4-bit chunks of the raw
  // value; the coder consumes that stream LIFO, so walking symbols backwards we emit the raw
  // chunks (last first), then nb, then the symbol.  Each emit writes at most one 32-bit word.
  uint32_t* ptr = ptr_;
  uint64_t x = x_;
  const EncSym* es = t.enc.data();
  const int32_t* len = t.length.data();
  const int32_t* off = t.offset.data();
  const int stride = t.stride;
  const uint32_t ntab = (uint32_t)t.n;
  for (int64_t i = n; i-- > 0;) {
    if ((size_t)(ptr - out_.data()) < 16) {
      ptr_ = ptr;
      grow();
      ptr = ptr_;
    }
    const int32_t ci = (int32_t)indexes[i];
    if ((uint32_t)ci >= ntab) throw std::runtime_error("rans: cdf index out of range");
    const int32_t max_value = len[ci] - 2;
    int32_t value = (int32_t)symbols[i] - off[ci];
    if ((uint32_t)value >= (uint32_t)max_value) {  // value < 0 or value >= max_value
      const uint32_t raw = value < 0 ? (uint32_t)(-2 * (int64_t)value - 1) : (uint32_t)(2 * ((int64_t)value - max_value));
      int32_t nb = 0;
      while (nb < 8 && (raw >> (nb * BYPASS_PRECISION)) != 0) ++nb;
      for (int32_t j = nb; j-- > 0;) enc_put_bits(x, ptr, (raw >> (j * BYPASS_PRECISION)) & MAX_BYPASS_VAL, BYPASS_PRECISION);
      enc_put_bits(x, ptr, (uint32_t)nb, BYPASS_PRECISION);
      value = max_value;
    }
    enc_put_sym(x, ptr, es[(int64_t)ci * stride + value]);
  }
  ptr_ = ptr;
  x_ = x;
}

template void RansEncoder::put_reverse<int32_t, int32_t>(const int32_t*, const int32_t*, int64_t, const CdfTables&);
template void RansEncoder::put_reverse<int16_t, uint8_t>(const int16_t*, const uint8_t*, int64_t, const CdfTables&);
template void RansEncoder::put_reverse<int32_t, uint8_t>(const int32_t*, const uint8_t*, int64_t, const CdfTables&);

std::string RansEncoder::flush() {
  if ((size_t)(ptr_ - out_.data()) < 2) grow();
  ptr_ -= 2;
  ptr_[0] = (uint32_t)(x_ >> 0);
  ptr_[1] = (uint32_t)(x_ >> 32);
  const size_t nbytes = (size_t)(end_ - ptr_) * sizeof(uint32_t);
  return std::string(reinterpret_cast<const char*>(ptr_), nbytes);
}

std::string rans_encode(const int32_t* symbols, const int32_t* indexes, int64_t n, const CdfTables& t) {
  RansEncoder e(n);
  e.put_reverse(symbols, indexes, n, t);
  return e.flush();
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

static std::atomic<int> g_narrow_limit{32767};
void set_narrow_limit(int lim) { g_narrow_limit.store(lim <= 0 || lim > 32767 ? 32767 : lim); }
int narrow_limit() { return g_narrow_limit.load(std::memory_order_relaxed); }

template <class I, class S>
bool RansDecoderState::decode(const I* indexes, int64_t n, const CdfTables& t, S* out) {
  constexpr uint64_t mask = (1ull << PRECISION) - 1;
  constexpr int SHIFT = PRECISION - CdfTables::LUT_BITS;
  const int32_t* len = t.length.data();
  const int32_t* off = t.offset.data();
  const uint64_t* lut = t.lut.data();
  const int32_t* cdfs = t.cdf.data();
  const CdfTables::Dom* dom = t.dom.data();
  const int stride = t.stride;
  const int32_t nhi = sizeof(S) < sizeof(int32_t) ? (int32_t)narrow_limit() : 0;  // the narrow range
  uint64_t state = state_;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t ci = (int32_t)indexes[i];
    if ((uint32_t)ci >= (uint32_t)t.n) throw std::runtime_error("rans: cdf index out of range");
    const uint32_t cum = (uint32_t)(state & mask);
    const CdfTables::Dom d = dom[ci];
    int32_t s;
    uint32_t start, freq;
    if (cum - d.start < d.freq) {  // the dominant symbol (unsigned: cum below start wraps to a miss)
      s = d.sym;
      start = d.start;
      freq = d.freq;
    } else {
      const uint64_t e = lut[((size_t)ci << CdfTables::LUT_BITS) + (cum >> SHIFT)];
      s = (int32_t)(e & 0xffff);
      if (e >> 63) {
        start = (uint32_t)(e >> 16) & 0xffff;
        freq = (uint32_t)(e >> 32) & 0x1ffff;
      } else {
        const int32_t* cdf = cdfs + (int64_t)ci * stride;
        const int32_t l = len[ci];
        while (s < l - 1 && (uint32_t)cdf[s + 1] <= cum) ++s;
        start = (uint32_t)cdf[s];
        freq = (uint32_t)(cdf[s + 1] - cdf[s]);
      }
    }
    const int32_t max_value = len[ci] - 2;
    if (s > max_value) throw std::runtime_error("rans: corrupt stream");
    uint64_t x = freq * (state >> PRECISION) + cum - start;
    if (x < RANS64_L) x = (x << 32) | get_word();
    state = x;
    int32_t value = s;
    if (value == max_value) {
      auto get_bits = [&](uint32_t nb) {
        uint64_t y = state;
        const uint32_t v = (uint32_t)(y & ((1u << nb) - 1));
        y >>= nb;
        if (y < RANS64_L) y = (y << 32) | get_word();
        state = y;
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
    const int32_t v = value + off[ci];
    if (sizeof(S) < sizeof(int32_t) && (v < -nhi - 1 || v > nhi)) {
      state_ = state;  // the caller resets to its mark and decodes again into a wider type
      return false;
    }
    out[i] = (S)v;
  }
  state_ = state;
  return true;
}
template bool RansDecoderState::decode<int32_t, int32_t>(const int32_t*, int64_t, const CdfTables&, int32_t*);

bool rans_decode_piece(RansDecoderState& d, const uint8_t* indexes, int64_t n, const CdfTables& t, int16_t* s16,
                       int32_t* s32) {
  const RansDecoderState::Mark m = d.mark();
  if (d.decode(indexes, n, t, s16)) return true;
  d.reset(m);
  d.decode(indexes, n, t, s32);
  return false;
}
template bool RansDecoderState::decode<uint8_t, int32_t>(const uint8_t*, int64_t, const CdfTables&, int32_t*);
template bool RansDecoderState::decode<uint8_t, int16_t>(const uint8_t*, int64_t, const CdfTables&, int16_t*);

void CdfTables::prepare() {
  enc.assign((size_t)n * stride, EncSym{~0ull, 1, 0, 0, 0});
  const size_t L = (size_t)1 << LUT_BITS;
  lut.assign((size_t)n * L, 0);
  dom.assign((size_t)n, Dom{0, 0, 0});
  for (int k = 0; k < n; ++k) {
    const int32_t* c = cdf.data() + (size_t)k * stride;
    const int len = length[k];
    if (len < 3 || len > stride || c[0] != 0 || c[len - 1] != (1 << PRECISION))
      throw std::runtime_error("rans: malformed cdf table");
    for (int v = 0; v + 1 < len; ++v) {
      if (c[v + 1] <= c[v]) throw std::runtime_error("rans: cdf not strictly increasing");
      enc[(size_t)k * stride + v] = make_enc_sym((uint32_t)c[v], (uint32_t)(c[v + 1] - c[v]));
    }
    // the dominant symbol among the regular ones (never the bypass escape len - 2)
    int best = 0;
    for (int v = 1; v < len - 2; ++v)
      if (c[v + 1] - c[v] > c[best + 1] - c[best]) best = v;
    // (only where it holds at least half the probability: a table whose dominant symbol is rarer would
    // mostly miss, and a test that mostly misses costs a mispredicted branch; freq 0 = never taken)
    const uint32_t bf = (uint32_t)(c[best + 1] - c[best]);
    dom[(size_t)k] = Dom{(uint32_t)c[best], bf >= (1u << (PRECISION - 1)) ? bf : 0u, best};
    int s = 0;
    const uint32_t width = 1u << (PRECISION - LUT_BITS);
    for (size_t b = 0; b < L; ++b) {
      const uint32_t lo = (uint32_t)(b << (PRECISION - LUT_BITS));
      while (s < len - 2 && (uint32_t)c[s + 1] <= lo) ++s;
      uint64_t e = (uint64_t)s;
      if ((uint32_t)c[s + 1] >= lo + width)  // the whole bucket lies inside symbol s
        e |= (1ull << 63) | ((uint64_t)(uint32_t)c[s] << 16) | ((uint64_t)(uint32_t)(c[s + 1] - c[s]) << 32);
      lut[(size_t)k * L + b] = e;
    }
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
