// Host build of the engine's raw DEFLATE decoder (automerge_amd/csrc/am_inflate_dec.h, the code the
// k_inflate_* kernels run per lane) for tests/test_inflate_host.py: reads length-prefixed streams,
// writes per stream a status byte (1 = inflated) and the length-prefixed output.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../automerge_amd/csrc/am_inflate_dec.h"

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* f = std::fopen(argv[1], "rb");
  FILE* g = std::fopen(argv[2], "wb");
  if (!f || !g) return 2;
  std::vector<uint16_t> T(amz::kSliceFast);
  uint32_t n;
  while (std::fread(&n, 4, 1, f) == 1) {
    // 64 bytes of slack after the stream, as the device arenas have (the bit reader's look-ahead)
    std::vector<uint8_t> in(n + 64 + 8, 0);
    uint8_t* p = in.data() + 1 + (n % 4);  // every alignment, as streams inside an arena have
    if (n && std::fread(p, 1, n, f) != n) return 2;
    // the short-stream decoder (register code search) and the long-stream one (one-lookup tables)
    for (int fast = 0; fast < 2; fast++) {
      const int64_t m = fast ? amz::inflate_raw<false, true>(p, n, nullptr, 0xFFFFFFF0u, T.data())
                             : amz::inflate_raw<false, false>(p, n, nullptr, 0xFFFFFFF0u, T.data());
      std::vector<uint8_t> out(m > 0 ? (size_t)m : 1);
      int64_t m2 = m;
      if (m >= 0)
        m2 = fast ? amz::inflate_raw<true, true>(p, n, out.data(), (uint64_t)m, T.data())
                  : amz::inflate_raw<true, false>(p, n, out.data(), (uint64_t)m, T.data());
      const uint8_t ok = (m >= 0 && m2 == m) ? 1 : 0;
      std::fwrite(&ok, 1, 1, g);
      const uint32_t k = ok ? (uint32_t)m : 0;
      std::fwrite(&k, 4, 1, g);
      if (k) std::fwrite(out.data(), 1, k, g);
    }
  }
  std::fclose(f);
  std::fclose(g);
  return 0;
}
