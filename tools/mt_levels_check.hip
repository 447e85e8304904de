// mt_levels_check.hip — host check of the MT19937 device draw's jump-job
// builder (build_levels / push_level in delta-node_amd/csrc/mt19937_device.hip,
// included here; no GPU needed): for substream counts S up to 300 and the
// boundary sizes up to 65537, for all four substream lengths (2^8 draws: direct levels only) and both
// generation modes, every window a generation wave starts from (1 .. S-1, or
// with backward generation the odd ones and S-1: mt_sub_forward) is produced
// exactly once (by a whole jump, or by the XOR of its parts) and no other
// window is, every source exists before its level, a workgroup's jobs share one
// source and one part (one table), part rows stay within the part-row region
// and cover the polynomial's words [0, 312) in order.
// Exit status 1 on any violation.
//
// build: hipcc -O1 -std=c++17 --offload-arch=gfx950 -I../include -I../delta-node_amd/csrc mt_levels_check.hip
#include "mt19937_device.hip"
#include <cstdio>
#include <map>
#include <set>
namespace dn { int set_error(int c, const char*, ...) { return c; } int device_cu_count() { return 256; }
uint64_t mt_jump_words() { return 0; } uint64_t mt_jump_max_subs() { return 262145; }
void mt_advance_window(const uint32_t*, uint64_t, uint32_t*) {}
const uint64_t* mt_direct_rows_l14(uint64_t, uint64_t*) { return nullptr; }
bool mt_xpow_mod(uint64_t, uint64_t*) { return false; } }
using namespace dn;
extern "C" uint64_t dn_m521_vec_bytes(uint64_t n) { return n; }
int check(uint64_t S, int ki, int back, bool rt = false) {
  const bool direct = S - 1 <= static_cast<uint64_t>(kMtDirectRows) || rt;
  // direct rows of this level: the tabulated D_s of length ki, or the runtime rows
  const int32_t dbase = rt ? kMtRtBase : kMtDirectBase + ki * kMtDirectRows;
  const int32_t dend = rt ? kMtRtBase + static_cast<int32_t>(kMtRtRows) : dbase + kMtDirectRows;
  Level LV[3];
  build_levels(S, ki, back, rt, LV);
  std::vector<const Level*> lv = {&LV[0], &LV[1], &LV[2]};
  std::vector<int> known(S + 1 + kPartRows + 8, 0);
  known[0] = 1;  // the caller's array; W_idx (level A's source) is window -1
  int bad = 0;
  for (size_t k = 0; k < lv.size(); ++k) {
    const Level& L = *lv[k];
    if (L.jobs.size() % L.W) { printf("S=%llu lvl %d jobs %% W\n", (unsigned long long)S, k); return 1; }
    std::map<int, std::tuple<int,int,int,int>> partw;  // row -> (src, poly, lo, hi)
    for (size_t g = 0; g < L.jobs.size(); g += L.W) {
      const JumpJob& j0 = L.jobs[g];
      if (j0.dst < 0) { printf("S=%llu lvl %d group starts with padding\n", (unsigned long long)S, k); return 1; }
      for (int w = 0; w < L.W; ++w) {
        const JumpJob& j = L.jobs[g + w];
        if (j.src != j0.src || (j.span & 0xffff) != (j0.span & 0xffff)) { bad++; }
        if (j.dst < 0) continue;
        if (j.src >= 0 && !known[j.src]) { printf("S=%llu lvl %d src %d unknown\n", (unsigned long long)S, k, j.src); return 1; }
        const int lo = j.span & 0xffff, hi = j.span >> 16;
        if (direct) {  // one level from W_idx, rows D_s of this length
          if (k != 0 || j.src != -1 || j.poly < dbase || j.poly >= dend) bad++;
          if (L.comb.empty() && j.poly != dbase + j.dst - 1) bad++;  // W(s) <- D_s
        } else if (ki >= kMtTabLens || j.poly < ki * kMtJumpRows || j.poly >= (ki + 1) * kMtJumpRows) {
          bad++;
        }
        if (L.comb.empty()) {
          if (lo != 0 || hi != kMtPolyWords) bad++;
          if (j.dst < 1 || (uint64_t)j.dst >= S || known[j.dst]) { printf("dst %d\n", j.dst); bad++; }
          known[j.dst] = 2;
        } else {
          if ((uint64_t)j.dst < S + 1 || (uint64_t)j.dst >= S + 1 + kPartRows || partw.count(j.dst)) bad++;
          partw[j.dst] = std::make_tuple(j.src, j.poly, lo, hi);
        }
      }
    }
    for (const CombineJob& c : L.comb) {
      if (c.dst < 1 || (uint64_t)c.dst >= S || known[c.dst]) bad++;
      int expect_lo = 0, src = -1, poly = -1;
      for (int p = 0; p < c.parts; ++p) {
        auto it = partw.find(c.first + p);
        if (it == partw.end()) { bad++; continue; }
        auto [s_, po, lo, hi] = it->second;
        if (p == 0) { src = s_; poly = po; }
        if (s_ != src || po != poly || lo != expect_lo) bad++;
        expect_lo = hi;
        partw.erase(it);
      }
      if (expect_lo != kMtPolyWords) bad++;
      if (direct && poly != dbase + c.dst - 1) bad++;  // W(s) <- D_s
      known[c.dst] = 2;
    }
    if (!partw.empty()) bad++;
    for (size_t i = 0; i < known.size(); ++i) if (known[i] == 2) known[i] = 1;
  }
  for (uint64_t s = 1; s < S; ++s)
    if (!known[s] != !mt_sub_forward(static_cast<uint32_t>(s), S, back)) bad++;
  if (bad) printf("S=%llu ki=%d back=%d bad=%d\n", (unsigned long long)S, ki, back, bad);
  return bad != 0;
}
int main() {
  int fails = 0;
  std::vector<uint64_t> Ss;
  for (uint64_t S = 1; S < 300; ++S) Ss.push_back(S);
  for (uint64_t S : {511ull, 512ull, 513ull, 1024ull, 1025ull, 2047ull, 2048ull, 2049ull, 4095ull, 4096ull, 4097ull, 4098ull, 5000ull, 8193ull, 16385ull, 20000ull, 65537ull})
    Ss.push_back(S);
  for (uint64_t S : Ss)
    for (int ki = 0; ki < kMtLens; ++ki) {
      if (ki >= kMtTabLens && S - 1 > static_cast<uint64_t>(kMtDirectRows)) continue;  // direct-only length
      fails += check(S, ki, 0) + check(S, ki, 1);
    }
  // the runtime direct level (2^14-draw substreams, backward generation, 65 < S <= 2049)
  for (uint64_t S : Ss)
    if (S - 1 > static_cast<uint64_t>(kMtDirectRows) && S - 1 <= kMtRtRows) fails += check(S, 2, 1, true);
  // summary for a few sizes
  for (uint64_t S : {2ull, 129ull, 513ull, 2049ull, 4097ull, 16385ull}) {
    Level L[3]; build_levels(S, 2, 1, false, L);
    printf("S=%6llu", (unsigned long long)S);
    for (int k = 0; k < 3; ++k) printf("  level %c: W=%d workgroups=%zu combines=%zu", "ACB"[k], L[k].W, L[k].jobs.size() / L[k].W, L[k].comb.size());
    printf("\n");
  }
  printf("fails %d\n", fails);
  return fails != 0;
}
