// Host check of the per-document workspace plan (automerge_amd/csrc/am_layout.h): every region
// offset and the total are 16-byte multiples for a sweep of document bounds, so the workspaces an
// exclusive scan of the totals places stay aligned (64-bit atomics of the global-mode hot set,
// 16-byte copies of the compaction). Built and run by tests/test_layout_host.py.
#include "am_layout.h"
#include <cstdio>
int main() {
  unsigned long bad = 0, n = 0;
  for (uint32_t R = 0; R < 700; R += 7)
    for (uint32_t E = 0; E < 700; E += 11)
      for (uint32_t P = 0; P < 3; P++) {
        DocBounds b{};
        b.R = R; b.E = E; b.C = R / 5 + 1; b.D = R / 7; b.A = 3; b.H = 2; b.N = R / 9; b.K = 2; b.AM = 5; b.ND = 4;
        b.P = P; b.S = R * 3 + 1; b.B = R * 11 + 3; b.span_lo = 5; b.span_hi = 5 + b.B;
        WsLayout L = ws_layout(b);
        n++;
        if ((L.total | L.hot_total | L.out | L.patch | L.pwire | L.dscr | L.etime) & 15) bad++;
      }
  printf("%lu %lu\n", n, bad);
  return bad != 0;
}
