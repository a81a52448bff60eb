"""compressai.ans placeholder: the reference's compress()/decompress() need the
C++ rANS coder; the fixture generator only drives forward() and the per-phase
symbol/index extraction, so these stubs just record calls."""


class BufferedRansEncoder:
    def encode_with_indexes(self, *a):
        self.args = a

    def flush(self):
        return b""


class RansDecoder:
    def set_stream(self, s):
        raise NotImplementedError("rANS decode is not available in the test shim")
