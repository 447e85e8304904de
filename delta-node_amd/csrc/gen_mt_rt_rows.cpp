// gen_mt_rt_rows.cpp — the build's generator of the MT19937 runtime direct
// jump rows D_1 .. D_kMtRtRows (csrc/host_gf2poly.cpp, mt_rt_rows_compute):
// writes them as raw little-endian uint64 words, then their two-word
// checksum (mt_rt_rows_checksum), to argv[1], which
// csrc/mt_rt_rows14.S embeds in the library (.incbin).  Linked against
// lib/host_gf2poly.o; run by delta-node_amd/Makefile.
#include <cstdint>
#include <cstdio>
#include <vector>

#include "dn_internal.hpp"

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: %s OUT.bin\n", argv[0]);
    return 2;
  }
  constexpr uint64_t kWords = 312;  // kMtPolyWords (csrc/mt19937_jump.inc)
  std::vector<uint64_t> rows(dn::kMtRtRows * kWords + 2);
  if (!dn::mt_rt_rows_compute(rows.data(), dn::kMtRtRows)) {
    std::fprintf(stderr, "gen_mt_rt_rows: no carry-less multiply on this host, or a row disagreed\n");
    return 1;
  }
  dn::mt_rt_rows_checksum(rows.data(), dn::kMtRtRows * kWords, rows.data() + dn::kMtRtRows * kWords);
  FILE* f = std::fopen(argv[1], "wb");
  if (!f || std::fwrite(rows.data(), sizeof(uint64_t), rows.size(), f) != rows.size() || std::fclose(f)) {
    std::fprintf(stderr, "gen_mt_rt_rows: cannot write %s\n", argv[1]);
    return 1;
  }
  return 0;
}
