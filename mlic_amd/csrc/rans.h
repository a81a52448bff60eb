// Host-native rANS entropy coder, byte-compatible with compressai 1.2.6's
// BufferedRansEncoder / RansDecoder (ryg_rans 64-bit state, 32-bit words, 16-bit CDF
// precision, 4-bit bypass escapes for out-of-range values), and pmf_to_quantized_cdf.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mlic {

struct EncSym {  // ryg_rans Rans64EncSymbol: exact division-free encode step
  uint64_t rcp_freq;
  uint32_t freq, bias, cmpl_freq, rcp_shift;
};

struct CdfTables {
  // table k: cdf[k * stride .. + length[k]]  (length includes the two sentinels, as compressai)
  std::vector<int32_t> cdf;
  std::vector<int32_t> length;
  std::vector<int32_t> offset;
  int stride = 0;
  int n = 0;
  bool empty() const { return n == 0; }
  // derived (prepare()): per-symbol encoder records and a 2^LUT_BITS decode bucket table
  static constexpr int LUT_BITS = 10;
  std::vector<EncSym> enc;       // [n][stride]
  // [n][1 << LUT_BITS] decode buckets: bit 63 set => the whole bucket decodes to one symbol and the
  // entry holds (symbol | start << 16 | freq << 32); else the low 16 bits are the first candidate
  std::vector<uint64_t> lut;
  // [n] the table's most probable symbol (largest frequency): its cdf start, its frequency and the symbol.
  // The decoder tests the state's cum against this one range first -- a 12-byte record per table, L1-
  // resident and independent of the state (loaded off the critical path) -- and only on a miss goes to the
  // bucket table (512 KB: L2).  At the bench's rates the dominant symbol is most of the stream.
  struct Dom {
    uint32_t start, freq;
    int32_t sym;
  };
  std::vector<Dom> dom;
  void prepare();
};

// Encodes symbols[i] with table indexes[i]; returns the byte string (little-endian u32 words).
std::string rans_encode(const int32_t* symbols, const int32_t* indexes, int64_t n, const CdfTables& t);

// The same coder over a stream given in pieces: rANS codes LIFO, so the pieces are handed over
// last first (put_reverse(piece k) for k = last .. 0), each walked backwards; flush() then returns
// exactly rans_encode() of the concatenation.  Lets the caller code an image's phases straight from
// the phase-major batch buffers without gathering them.
class RansEncoder {
 public:
  explicit RansEncoder(int64_t n_hint);
  // S: int32_t / int16_t symbols, I: int32_t / uint8_t table indexes (the narrow forms are what crosses
  // PCIe: a scale index is < 64, a symbol almost always fits 16 bits)
  template <class S, class I>
  void put_reverse(const S* symbols, const I* indexes, int64_t n, const CdfTables& t);
  std::string flush();

 private:
  std::vector<uint32_t> out_;
  uint32_t* end_;
  uint32_t* ptr_;
  uint64_t x_ = 1ull << 31;  // RANS64_L
  void grow();
};

// The narrow-transfer range test knob (mlic_set_kernel_option("narrow_limit", L)): symbols outside
// [-L - 1, L] take the int32 fallback on both sides (the encoder's *ovf copy, the decoder's re-decode into
// int32); default / L <= 0 / L > 32767: the int16 range.  Bitstreams are the same bytes whatever L is;
// the knob exists so that the fallback paths run in tests.
void set_narrow_limit(int lim);
int narrow_limit();

class RansDecoderState;
// one piece (a phase of one image) of the decompress path's narrow decode: into s16 when every value fits
// the narrow range (returns true), else reset to the piece's start and decoded into s32 (returns false)
bool rans_decode_piece(RansDecoderState& d, const uint8_t* indexes, int64_t n, const CdfTables& t, int16_t* s16,
                       int32_t* s32);

class RansDecoderState {
 public:
  void set_stream(const uint8_t* data, size_t nbytes);
  // decodes n symbols with the given table indexes; false (output incomplete, state past it) when a
  // value does not fit S -- reset() to a mark() taken before and decode again into int32_t
  template <class I, class S>
  bool decode(const I* indexes, int64_t n, const CdfTables& t, S* out);
  struct Mark {
    size_t pos;
    uint64_t state;
  };
  Mark mark() const { return {pos_, state_}; }
  void reset(const Mark& m) {
    pos_ = m.pos;
    state_ = m.state;
  }

 private:
  std::vector<uint32_t> words_;
  size_t pos_ = 0;
  uint64_t state_ = 0;
  uint32_t get_word();
};

std::vector<uint32_t> pmf_to_quantized_cdf(const float* pmf, int n, int precision);

}  // namespace mlic
