// stream.hip — the planned expansion of the big nets (default for L1 = 3072 / 1024).
//
// The incremental evaluation of every parent and every legal child (SURVEY.md §8a
// rows a13-a17, "children are derived from the parent accumulator by incremental
// add/sub deltas") in two kernels:
//
//   plan_kernel         one wave per block of consecutive parents (a game): turns the
//                       block's slots [parent, its children, next parent, ...] into
//                       two lists of row entries (one per absolute perspective) and a
//                       descriptor per 16-slot tile, in HBM.  Every decision that is
//                       sequential inside a block is made here: the sibling cache, the
//                       chain (parent p + 1 starts from parent p's child that is its
//                       position: that child is evaluated last among its siblings and its
//                       accumulators become the parent accumulators), the king cache
//                       (Stockfish's AccumulatorCaches analog: a king-move refresh starts
//                       from the accumulator the block last computed for that perspective
//                       and king square, plus the placement difference), the list balance,
//                       and every PSQT sum (PSQT never enters the row stream).
//   stream_eval_kernel  one workgroup per block: each perspective group of waves walks
//                       its list with a 4-deep register ring of row loads, transforms at
//                       each slot's last entry into the LDS tile, and after each tile
//                       all waves run fc_0 as int8 MFMAs; one wave per bucket finishes
//                       fc_1 / fc_2 and writes the outputs while the others stream on.
//
// Entry (u64, built by the plan kernel in the form the stream consumes):
//   lo = the row's byte offset: an FT row, the zero row, or (bit 31, SCR) a row of the
//        workgroup's scratch slot counted from its first row (2 + 64 h + ksq: the
//        king-cache row of (h, ksq)); the workgroup adds its slot's offset (the FT table is
//        < 2^28 bytes, so bit 31 is free)
//   hi = [15:0] the 16-bit multiplier of the row (1 add, 0xFFFF subtract, 0 no-op; a
//        store-only KST entry loads the zero row and has its target scratch row here),
//        [17:16] the init before the entry (0 none, 1 ZERO: acc = row, 2 PACC: acc = parent
//        - row, saved as the sibling base, 3 BASE: acc = base +- row), [18] LAST entry of its
//        slot, [19] X (PAR_E or KST), [20] PAR_E (the slot's accumulator becomes pacc: a
//        parent, or the child that is the next parent), [21] KST (store the slot's
//        accumulator to the scratch row of this entry), [31:22] where the slot's features go
//        in the LDS tile: (slot in tile) * xu + (side) * hu, side 0 the perspective to move,
//        in the stream's units (plan_kernel's xu / hu: 16-B units of the tile row XS and of
//        the half LC / 2 for the column-sliced and 1024-wide streams; slot * 2 + side for
//        the whole-row 3072 stream)
// Round 6: each test the stream makes is one bit or one field of hi, nested so that an entry
// runs only the tests of its kind (round 5's decode ran ~25 scalar instructions per entry, the
// scalar unit's issue being the larger part of the stream's issue floor), and the LDS address
// of the features is a shift of hi.
// The ring issues a row load 4 entries before it
// consumes it, so an entry that loads a scratch row sits at least GN_SCR_GAP (= 4) entries
// after the last store to scratch in its list (no-op entries are inserted when needed): the
// load is then issued after the store, by the same lanes (kernels.h: why that suffices).
// The ring runs across tiles.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "device_util.h"
#include "kernels.h"

#ifndef GN_PLAN_WPE
#define GN_PLAN_WPE 4 // <= 128 VGPRs, no spills (round 3: 3 waves at 168 VGPRs beat 4 with spills; round 4 fits 4)
#endif
#ifndef GN_SLICE_WPE // the column-sliced stream (2-wave workgroups): 4 waves per SIMD (<= 128 VGPRs; LDS holds
#define GN_SLICE_WPE 4 // 8 workgroups per CU).  Round 5's weight cache and partial-sum prefetch need 126 at that
#endif                 // bound (130 unbounded, i.e. 3 per SIMD).  (Round 4: with the finish in the last slice,
                       // 125 + 8 AGPRs, 3 per SIMD 157.1 ms, forced to 4 160.4 ms)
#define GN_PART_N GN_PART_SLICES
#ifndef GN_WCACHE // the sliced stream's per-wave fc_0 weight cache (0: weights loaded at each layer stack)
#define GN_WCACHE 1
#endif
#ifndef GN_EXPAND_WPE
#define GN_EXPAND_WPE (GN_RING == 4 ? 5 : 4)
#endif
#define GN_STR2(x) #x
#define GN_STR(x) GN_STR2(x)

#ifdef GN_STREAM_PROF
// diagnostics build only: per-phase s_memtime cycles summed over waves, and list balance
__device__ unsigned long long gn_sp[8]; // [0] stream [1] barrier wait [2] layer stack [3] tiles
                                       // [4] sum max(n0, n1) [5] sum n0 + n1 [6] / [7] no-op entries (scratch order / tile end)
#define SP_T() __builtin_amdgcn_s_memtime()
#define SP_ADD(k, v) atomicAdd(&gn_sp[k], (unsigned long long)(v))
#else
#define SP_T() 0ull
#define SP_ADD(k, v) (void)(v)
#endif
#ifdef GN_PLAN_PROF
// diagnostics build only: plan_kernel cycles (s_memtime) per section, summed over waves:
// [0] parent setup [1] slot descriptors, prefix sums, PSQT, the parent rows [2] delta puts, tile ends
// [3] king-move jobs
__device__ unsigned long long gn_pp[4];
#define PP_T() __builtin_amdgcn_s_memtime()
#define PP_ADD(k, v) atomicAdd(&gn_pp[k], (unsigned long long)(v))
#else
#define PP_T() 0ull
#define PP_ADD(k, v) (void)(v)
#endif
#ifdef GN_XCD_PROF
// diagnostics build only: per XCD, [x] the last workgroup end and [8 + x] the first start
// (s_memrealtime, 100 MHz, chip-wide), [16 + x] entries streamed, [24 + x] workgroups
__device__ unsigned long long gn_xp[32] = {0, 0, 0, 0, 0, 0, 0, 0, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull, ~0ull};
#endif

#ifdef GN_FAULT_PLAN_BLOCK
// fault-injection build only (fishnet_amd/build.py FAULT_LIB; tests/test_gpu_parity.py
// ::test_plan_overflow_fails_the_call_then_recovers): armed once per process
__device__ int gn_fault_armed = 1;
#endif

namespace gn {
namespace ps {
// (bits 16-17 of the header word: the kind field HZ / HP / HB below)
constexpr uint32_t H_LAST = 1u << 18, H_X = 1u << 19,
                   H_PAR_E = H_X | 1u << 20, H_KST = H_X | 1u << 21, H_LDS_SH = 22;
constexpr uint32_t L_SCR = 1u << 31; // (in lo)
// Each put site knows its entry's kind, so hi is a constant mask or'd with the slot / side
// field (round 3 built a u32 entry and decoded it per put: ~25 VALU per entry in an
// issue-bound kernel).
constexpr uint32_t M_ADD = 1u, M_SUB = 0xFFFFu;
constexpr uint32_t HZ = 1u << 16, HP = 2u << 16, HB = 3u << 16;
// the slot's LDS field (xu / hu: plan_kernel's arguments, see above)
__device__ __forceinline__ uint32_t hs(int slot, int side, uint32_t xu, uint32_t hu) {
  return ((uint32_t)slot * xu + (uint32_t)side * hu) << H_LDS_SH;
}
// a stream whose tile rows (XS bytes) and halves (LC / 2) are whole 16-B units that fit the
// 10-bit field for 16 slots takes its LDS offset as field << 4; otherwise the field is slot * 2
// + side
constexpr bool lds_field16(int XS, int LC) {
  return XS % 16 == 0 && (LC / 2) % 16 == 0 && 15 * (XS / 16) + LC / 32 < 1024;
}
#ifndef GN_SLICE_XPAD // A/B: LDS bytes added per tile row of the sliced stream (fewer workgroups per CU)
#define GN_SLICE_XPAD 0
#endif
// the stream's LDS tile row (bytes) for L1 / SL columns, and the plan's (xu, hu) for it
constexpr int tile_xs(int L1, int SL) { return L1 / SL + 16 + (SL > 1 ? GN_SLICE_XPAD : 0); }
constexpr uint32_t field_xu(int L1, int SL) {
  return lds_field16(tile_xs(L1, SL), L1 / SL) ? (uint32_t)tile_xs(L1, SL) / 16 : 2u;
}
constexpr uint32_t field_hu(int L1, int SL) { return lds_field16(tile_xs(L1, SL), L1 / SL) ? (uint32_t)(L1 / SL) / 32 : 1u; }
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
} // namespace ps

// ------------------------------------------------------------------- plan --
constexpr int PLAN_WAVES = GN_FRONT_WG / 64; // one block per wave, no workgroup barriers
template <int L1>
__global__ void __launch_bounds__(GN_FRONT_WG) __attribute__((amdgpu_waves_per_eu(GN_PLAN_WPE)))
    plan_kernel(NetDevice net, const gn_board *__restrict__ parents, const uint64_t *__restrict__ offsets,
                const ChildDelta *__restrict__ deltas, const uint8_t *__restrict__ need_parent,
                const uint8_t *__restrict__ need_child, const uint8_t *__restrict__ next_slot, uint32_t np, uint32_t K,
                uint32_t b0, uint32_t b1, int kc, const uint64_t *__restrict__ eoff, uint64_t *__restrict__ ent, TileDesc *__restrict__ tiles,
                uint32_t *__restrict__ btiles, unsigned long long *__restrict__ rows_out,
                unsigned long long *__restrict__ pads_out, uint32_t *__restrict__ err, int2 *__restrict__ pinfo,
                uint32_t xu, uint32_t hu) {
  using namespace ps;
  __shared__ uint32_t ksnap[PLAN_WAVES][128][8]; // per wave: placement (64 nibbles) of each king-cache row
  __shared__ uint16_t prow_s[PLAN_WAVES][2][32];
  __shared__ uint32_t jrow_s[PLAN_WAVES][4][64]; // per wave: the first four jobs' (row + 1) | pos << 16 | cpc << 24, lane = square
  // (w via readfirstlane: the compiler then knows that blk, p and every bound derived from them
  // are wave-uniform, so they live in SGPRs and their branches are scalar)
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t blk = b0 + blockIdx.x * PLAN_WAVES + (uint32_t)w; // this launch plans blocks [b0, b1)
  if (blk >= b1) return; // the whole wave (no workgroup barriers in this kernel)
  const __amdgpu_buffer_rsrc_t pst = __builtin_amdgcn_make_buffer_rsrc(
      (void *)net.psqt, 0, (int)((size_t)PSQT_BUCKETS * FT_ROWS * 4), 0x00020000);
  auto psqt = [&](uint32_t row, int bucket) -> int32_t { // bucket-major copy (L2-resident)
#ifdef GN_AB_PLAN_NOPSQT // timing diagnostics only (wrong PSQT): the plan without its PSQT loads
    return (int32_t)(row + bucket);
#endif
    return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(pst, (bucket * (uint32_t)FT_ROWS + row) * 4, 0, 0);
  };
  const uint32_t pbeg = blk * K, pend = pbeg + K < np ? pbeg + K : np;
  const uint64_t us_b = pbeg + offsets[pbeg];
  const uint64_t rbeg = eoff[pbeg] + (uint64_t)ENT_SPARE * blk, rend = eoff[pend] + (uint64_t)ENT_SPARE * (blk + 1);
  uint2 *E = reinterpret_cast<uint2 *>(ent + rbeg); // list 0 from E[0] up, list 1 from E[rtot - 1] down
  const uint32_t rtot = (uint32_t)(rend - rbeg); // the block's entry region (both lists; < 2^32)
  uint32_t bad = 0;                  // this lane's error bits (reported once per wave)
  // a block's tiles: <= ceil(slots / 16) + one bucket cut per parent (a parent's own slots hold
  // <= 2 buckets, so a tile is cut at most once per parent), hence this base
  TileDesc *T = tiles + us_b / 16 + (uint64_t)(K + 2) * blk;
  uint32_t safe0 = 0, safe1 = 0; // first index of each list at which a scratch row may be loaded
  constexpr uint32_t RS = ft_row_stride(L1);
  constexpr uint32_t LO_BIAS = (uint32_t)FT_BIAS_ROW * RS, LO_ZERO = (uint32_t)ZERO_ROW * RS;
  auto lo_scr = [](uint32_t r) -> uint32_t { return ((uint32_t)FT_ROWS + r) * RS | L_SCR; }; // scratch row r
  // entry i of list g: the row at byte offset lo, hi = multiplier + flags (see above)
  // One SGPR base and an unsigned 32-bit byte offset for both lists: the store is the base + a
  // VGPR offset, no 64-bit address arithmetic per entry.  Entries are only ever put below their
  // list's final length, so the final check (len0 + len1 <= rtot) covers every put; the clamp
  // keeps an overflow (which fails the call) inside the region.
  const uint32_t rlast = rtot - 1;
  auto put = [&](int g, uint32_t i, uint32_t lo, uint32_t hi) {
    // a scratch-row load must sit GN_SCR_GAP entries after the list's last scratch store
    if ((lo & L_SCR) && i < (g ? safe1 : safe0)) bad |= 4u;
    const uint32_t ic = i < rlast ? i : rlast;
    const uint32_t x = g ? rlast - ic : ic;
    *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(E) + (x << 3)) = make_uint2(lo, hi);
  };
  // king-cache row state, lane = king square, one register per perspective: bit 0 the row holds an
  // accumulator, bit 1 the list that stored it (v_readlane / a select: no LDS round trip)
  uint32_t ks0 = 0, ks1 = 0;
  auto kstate_of = [&](int hh, int ksq) -> int { return __builtin_amdgcn_readlane((int)(hh ? ks1 : ks0), ksq); };
  auto kstate_set = [&](int hh, int ksq, int v) {
    if (hh) ks1 = lane == ksq ? (uint32_t)v : ks1;
    else ks0 = lane == ksq ? (uint32_t)v : ks0;
  };
  uint16_t(*prow)[32] = prow_s[w];
  uint32_t len0 = 0, len1 = 0, tile_k = 0, p_first = pbeg, u_fill = 0, t_first = 0, tile_bm = 0;
  unsigned long long pp_a = 0, pp_b = 0, pp_c = 0, pp_d = 0; // GN_PLAN_PROF: section cycles
  int t_fill = 0, carried = 0;
  uint32_t rows = 0, pads = 0, fpads = 0; // (per block: < 2^32)
  auto pad_to = [&](int g, uint32_t target) { // no-op entries up to target (lane-parallel, < 64)
    uint32_t &len = g ? len1 : len0;
    if (len < target) {
      pads += target - len;
      if ((uint32_t)lane < target - len) put(g, len + lane, LO_BIAS, 0u); // (no-op: multiplier 0)
      len = target;
    }
  };

  // a field of tile k of the block by a 32-bit byte offset from the block's first tile (the
  // stores are then an SGPR base + a VGPR offset)
  char *const Tb = reinterpret_cast<char *>(T);
  auto tf = [&](uint32_t k, uint32_t field) -> char * { return Tb + (k * (uint32_t)sizeof(TileDesc) + field); };
  auto flush = [&]() {
    // (the lists need no padding at a tile's end: the stream enters and leaves its ring
    // revolutions at any entry)
    if (lane >= t_fill && lane < 16) *tf(tile_k, offsetof(TileDesc, meta) + lane) = 0;
    if (lane == 0) *reinterpret_cast<uint4 *>(tf(tile_k, 0)) = make_uint4(len0, len1, p_first, t_first);
    ++tile_k, t_fill = 0, tile_bm = 0;
  };

  // ---- a parent's inputs are loaded while the previous parent is planned, so that a parent
  // waits for memory about twice (its inputs; then all its PSQT rows at once) instead of once
  // per dependent load: lanes 0..6 the board's first 28 bytes (bd), lane 1 + c child c's delta
  // (a, b, c, d its rows, m its meta, nd the aligned word holding its need_child byte), lane 0
  // m / nd the words holding next_slot[p] / need_parent[p].  Children beyond the 63rd are
  // loaded in their own pass.  The values stay as loaded, with no branch around a load (any
  // arithmetic on them, or a copy where two paths meet, would wait for them here); an absent
  // array is read from the board instead and ignored.  (The library allocates its byte arrays in
  // whole 16-B units, so the aligned word holding a last byte is inside the allocation.)
  struct In {
    uint32_t bd, a, b, c, d, m, nd;
  };
  auto word = [](const uint8_t *b) { return *reinterpret_cast<const uint32_t *>((uintptr_t)b & ~(uintptr_t)3); };
  auto byte_of = [](uint32_t wv, const uint8_t *b) { return (wv >> (8 * ((uintptr_t)b & 3))) & 0xFFu; };
  auto fetch = [&](uint32_t p) -> In {
    const uint64_t off = offsets[p];
    const uint32_t nch = (uint32_t)(offsets[p + 1] - off);
    const uint8_t *any = reinterpret_cast<const uint8_t *>(parents + p);
    In x = {0, 0, 0, 0, 0, 0, 0};
    if (lane < 7) x.bd = reinterpret_cast<const uint32_t *>(parents + p)[lane];
    if (lane == 0) {
      x.m = word(next_slot ? next_slot + p : any);
      x.nd = word(need_parent ? need_parent + p : any);
    } else if ((uint32_t)lane - 1 < nch) {
      const uint32_t *src = reinterpret_cast<const uint32_t *>(deltas + off + lane - 1);
      x.a = src[0], x.b = src[1], x.c = src[2], x.d = src[3], x.m = src[4];
      x.nd = word(need_child ? need_child + off + lane - 1 : any);
    }
    return x;
  };
  In xd = {0, 0, 0, 0, 0, 0, 0};
  if (pbeg < pend) xd = fetch(pbeg);
  for (uint32_t p = pbeg; p < pend; ++p) {
    unsigned long long pp_t = PP_T();
    const uint64_t off = offsets[p];
    const int nch = (int)(offsets[p + 1] - off), total = 1 + nch;
    gn_board pb = {};
    {
      uint32_t pw[7];
#pragma unroll
      for (int i = 0; i < 7; ++i) pw[i] = (uint32_t)__builtin_amdgcn_readlane((int)xd.bd, i);
      pb.occ = (uint64_t)pw[0] | (uint64_t)pw[1] << 32;
      __builtin_memcpy(pb.pc, &pw[2], 16);
      pb.stm_ep = (uint8_t)pw[6];
    }
    const uint32_t f0 =
        (need_parent ? byte_of((uint32_t)__builtin_amdgcn_readlane((int)xd.nd, 0), need_parent + p) : 1u) |
        (next_slot ? byte_of((uint32_t)__builtin_amdgcn_readlane((int)xd.m, 0), next_slot + p) : 255u) << 8;
    const bool pre = total <= 64; // the parent's slots are one pass, its inputs prefetched
    const int P = wave_features(pb, prow[0], prow[1], lane);
    ps::wave_sync();
    int want = 0;
    if (pre) want = lane == 0 ? (int)(f0 & 0xFF) : lane < total ? (int)(need_child ? byte_of(xd.nd, need_child + off + lane - 1) : 1u) : 0;
    else
      for (int q = lane; q < total; q += 64)
        want |= q == 0 ? (int)(f0 & 0xFF) : (need_child ? need_child[off + q - 1] : 1);
    const bool live = __ballot(want) != 0 && P != 0;
    const int have = live ? carried : 0;
    carried = 0;
    const int stm = pb.stm_ep >> 7;
    const int bp = P ? (P - 1) / 4 : 0, b2 = P >= 2 ? (P - 2) / 4 : bp;
    // parent PSQT per perspective at the two buckets its children can have (lane = (h, row)):
    // loaded in pass 0 with the slots' rows, then summed
    int32_t pp[2][2] = {{0, 0}, {0, 0}}, pa = 0, pb2 = 0;
    int nxq = -1; // slot (1 + child index) of the child that is the next parent
    if (live && K > 1 && p + 1 < pend) {
      const int ns = (int)(f0 >> 8);
      if (ns != 255 && ns < nch) {
        const bool nd = ns + 1 < 64 ? (!need_child || byte_of((uint32_t)__builtin_amdgcn_readlane((int)xd.nd, ns + 1), need_child + off + ns) != 0)
                                    : (!need_child || need_child[off + ns]);
        if (nd) nxq = ns + 1;
      }
    }
    carried = nxq > 0;
    // the child that is the next parent is evaluated last among its siblings (its accumulators
    // then become the parent accumulators the next parent starts from): processing position q
    // (1..nch) takes child ci(q), the others keep their order
    auto child_of = [&](int q) -> int {
      const int c = q - 1;
      return nxq > 0 && c >= nxq - 1 ? (c < nch - 1 ? c + 1 : nxq - 1) : c;
    };
    const int nxpos = nxq > 0 ? nch : -1;
    int ckey0 = -1, ckey1 = -1; // sibling keys carried across this parent's segments
    // ---- a refreshed parent starts from the king cache when the block last computed an
    // accumulator for this perspective and king square (Stockfish's AccumulatorCaches for
    // a refresh): cache row + the placement differences; either way the parent's
    // accumulator is stored back to that row (a sibling batch, as in a depth-2 expansion,
    // then refreshes every parent from its predecessor's row).  Per perspective hh, in
    // list hh (its entries end with PAR_E: list hh's parent register).
    int pnd[2] = {-1, -1};        // entries between the cache row and the store (< 0: full refresh)
    bool pst[2] = {false, false}; // the refresh is stored to the cache row
    int pkq[2] = {0, 0};          // the perspective's king square
    // the cached placement's piece on this lane's square and the differences to ppc
    auto cache_diff = [&](int kci, int pc, int &spc, uint64_t &bs, uint64_t &ba) {
      spc = (int)((ksnap[w][kci][lane >> 3] >> (4 * (lane & 7))) & 15);
      bs = __ballot(spc != pc && spc != 0), ba = __ballot(spc != pc && pc != 0);
    };
    const int ppc = live ? lane_piece(pb, lane) : 0; // the parent's piece on this lane's square
    if (live && !have && kc) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const uint64_t kb = __ballot(ppc == make_piece(hh, KING));
        const int ksq = kb ? __builtin_ctzll(kb) : 0, kci = 64 * hh + ksq;
        pkq[hh] = ksq;
        const int kst = kstate_of(hh, ksq);
        pst[hh] = kb != 0 && (kst == 0 || ((kst >> 1) & 1) == hh); // the row is unused or list hh's
        if (pst[hh] && (kst & 1)) {
          int spc;
          uint64_t bs, ba;
          cache_diff(kci, ppc, spc, bs, ba);
          const int nd = popcnt(bs) + popcnt(ba);
          if (nd < P) pnd[hh] = nd;
        }
      }
    }

    pp_a += PP_T() - pp_t;
    // ---- the parent's slots (lane = slot) in passes of up to 64 (one pass unless the parent has
    // more than 63 children).  A pass fills the open tile (cut early where a third layer-stack
    // bucket would enter it) and as many new 16-slot tiles as its slots need.  A tile's region
    // of each list is [its delta entries: the parent's and the delta perspectives', slot order]
    // then [its king-move refresh entries, slot order]: the king-move jobs run first, tile by
    // tile (each tile's delta region is reserved when the cursor reaches it), then every lane
    // puts its delta entries at once.
    for (int q0 = 0; q0 < total; q0 += 64) {
      pp_t = PP_T();
      const int n_in = total - q0 < 64 ? total - q0 : 64;
      const int q = q0 + lane;
      // ---- descriptor of this lane's slot
      int vld = 0, cst = 0, cnt = 1, kinds = 0, n0 = 0, n1 = 0, s0 = 0, s1 = 0;
      uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
      In y = {0, 0, 0, 0, 0, 0, 0};
      if (pre) { // (pass 0) the prefetched inputs in processing order: slot q = child child_of(q)
        const int sl = q >= 1 && q < total ? child_of(q) + 1 : 0;
        y.a = (uint32_t)__shfl((int)xd.a, sl), y.b = (uint32_t)__shfl((int)xd.b, sl);
        y.c = (uint32_t)__shfl((int)xd.c, sl), y.d = (uint32_t)__shfl((int)xd.d, sl);
        y.m = (uint32_t)__shfl((int)xd.m, sl), y.nd = (uint32_t)__shfl((int)xd.nd, sl);
      }
      __builtin_amdgcn_sched_barrier(0); // (the shuffles' wait must not cover the loads below)
      if (q0 == 0 && p + 1 < pend) xd = fetch(p + 1); // the next parent's inputs
      if (q0 == 0 && live && (lane & 31) < P)
        pa = psqt(prow[lane >> 5][lane & 31], bp), pb2 = psqt(prow[lane >> 5][lane & 31], b2);
      if (lane < n_in && live) {
        if (q == 0) {
          vld = (int)(f0 & 0xFF);
          cst = stm, cnt = P, kinds = 3 | 3 << 2;
        } else if ((vld = pre ? (int)(need_child ? byte_of(y.nd, need_child + off + child_of(q)) : 1u) : need_child ? need_child[off + child_of(q)] : 1)) {
          uint32_t meta;
          if (pre) {
            w0 = y.a, w1 = y.b, w2 = y.c, w3 = y.d, meta = y.m;
          } else {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(deltas + off + child_of(q));
            w0 = src[0], w1 = src[1], w2 = src[2], w3 = src[3], meta = src[4];
          }
          cst = (meta >> 10) & 1;
          cnt = (meta >> 14) & 63;
          if (meta & (1u << 8)) kinds |= 2, n0 = cnt + 1;
          else kinds |= 1, s0 = meta & 3, n0 = s0 + ((meta >> 2) & 3);
          if (meta & (1u << 9)) kinds |= 2 << 2, n1 = cnt + 1;
          else kinds |= 1 << 2, s1 = (meta >> 4) & 3, n1 = s1 + ((meta >> 6) & 3);
        }
      }
      const bool in = lane < n_in;
      const int bk = (cnt - 1) / 4;
      const bool ref0 = (kinds & 3) == 2, ref1 = (kinds >> 2) == 2;
      // ---- every PSQT load of the pass before any of its waits (a wait for a load also waits
      // for the stores issued before it, so loads go out first): the delta rows of each slot,
      // and the first four king-move jobs' rows (lane = square); the rest of the jobs later
      int32_t dq[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
      if (in && live) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if ((hh ? kinds >> 2 : kinds & 3) == 1) {
            const uint32_t lo2 = hh ? w2 : w0, hi2 = hh ? w3 : w1;
            const int s = hh ? s1 : s0, n = hh ? n1 : n0;
            const uint32_t i0 = lo2 & 0xFFFF, i1 = lo2 >> 16, i2 = hi2 & 0xFFFF, i3 = hi2 >> 16;
            const uint32_t r1 = s >= 2 ? i1 : i2, r2 = s >= 2 ? i2 : i3;
            dq[hh][0] = psqt(ft_row(i0), bk), dq[hh][1] = psqt(ft_row(r1), bk);
            if (n > 2) dq[hh][2] = psqt(ft_row(r2), bk);
            if (n > 3) dq[hh][3] = psqt(ft_row(i3), bk);
          }
        }
      }
      uint64_t jm = __ballot(in && live && vld && (ref0 || ref1)), jrest = jm;
      int32_t jv[4] = {0, 0, 0, 0};
      int jl[4] = {-1, -1, -1, -1}; // their slot lanes
      auto job_rows = [&](int l, int &row, int &pos, int &cpc) { // job l's row on this lane's square
        const int hh = __builtin_amdgcn_readlane((int)ref1, l);
        const uint32_t sq01 = (uint32_t)__builtin_amdgcn_readlane((int)(hh ? w2 : w0), l),
                       sq23 = (uint32_t)__builtin_amdgcn_readlane((int)(hh ? w3 : w1), l);
        row = king_move_row_pc(ppc, hh, sq01 & 0xFFFF, (int)(sq01 >> 16), sq23 & 0xFFFF, sq23 >> 16, lane, pos, cpc);
      };
      auto job_row_psqt = [&](int l, int row) -> int32_t { // its PSQT row
        const int cn = __builtin_amdgcn_readlane(cnt, l);
        return row >= 0 ? psqt((uint32_t)row, (cn - 1) / 4) : 0;
      };
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (jrest) {
          const int l = __builtin_ctzll(jrest);
          jrest &= jrest - 1;
          int row, pos, cpc;
          job_rows(l, row, pos, cpc);
          jv[u] = job_row_psqt(l, row), jl[u] = l;
          jrow_s[w][u][lane] = (uint32_t)(row + 1) | (uint32_t)pos << 16 | (uint32_t)cpc << 24; // (for the job loop)
        }
      }
      // (the slot bookkeeping below runs while the PSQT loads are in flight)
      // ---- tiles of the pass: the open tile takes c1 slots, then tiles of 16
      const uint32_t mybit = in && live && vld ? 1u << bk : 0u;
      const uint32_t bits = scan_or(mybit);
      const uint64_t ok = __ballot(!in || __builtin_popcount(tile_bm | bits) <= 2);
      int lead = ok == ~0ull ? 64 : __builtin_ctzll(~ok);
      if (lead == 0) { // the open tile holds two other buckets: close it; a fresh tile takes every
        flush();       // slot of a parent (its slots hold <= 2 buckets: P and P - 1 pieces)
        if (__ballot(in && __builtin_popcount(bits) > 2)) bad |= 1u; // cannot happen; reported
        lead = 64;
      }
      if (t_fill == 0) p_first = p, t_first = u_fill;
      const int tf0 = t_fill, room = 16 - tf0;
      const int c1 = room < lead ? (room < n_in ? room : n_in) : (lead < n_in ? lead : n_in);
      const int tix = lane < c1 ? 0 : 1 + (lane - c1) / 16;        // this slot's tile, from tk0
      const int t = lane < c1 ? tf0 + lane : (lane - c1) % 16;     // its slot in that tile
      const int ntp = n_in <= c1 ? 1 : 1 + (n_in - c1 + 15) / 16; // tiles the pass touches
      const uint32_t tk0 = tile_k;
      if (!in) vld = 0, kinds = 0, n0 = n1 = s0 = s1 = 0, w0 = w1 = w2 = w3 = 0;
      // ---- sibling cache: a delta child whose from-row equals the previous delta child's (in
      // the same list) starts from the cached (parent - from-row) and drops that entry
      const int key0 = (kinds & 3) == 1 ? (int)(w0 & 0xFFFF) : -1;
      const int key1 = (kinds >> 2) == 1 ? (int)(w2 & 0xFFFF) : -1;
      const uint64_t km0 = __ballot(key0 >= 0), km1 = __ballot(key1 >= 0), lt = (1ull << lane) - 1;
      const int pk0 = __shfl(key0, (km0 & lt) ? 63 - __builtin_clzll(km0 & lt) : 0);
      const int pk1 = __shfl(key1, (km1 & lt) ? 63 - __builtin_clzll(km1 & lt) : 0);
      const bool hit0 = key0 >= 0 && key0 == ((km0 & lt) ? pk0 : ckey0);
      const bool hit1 = key1 >= 0 && key1 == ((km1 & lt) ? pk1 : ckey1);
      if (km0) ckey0 = __builtin_amdgcn_readlane(key0, 63 - __builtin_clzll(km0));
      if (km1) ckey1 = __builtin_amdgcn_readlane(key1, 63 - __builtin_clzll(km1));
      if (q0 == 0 && live) {
        const int a = (int)scan_add((uint32_t)pa), b = (int)scan_add((uint32_t)pb2);
        pp[0][0] = __builtin_amdgcn_readlane(a, 31), pp[0][1] = __builtin_amdgcn_readlane(b, 31);
        pp[1][0] = wadd(__builtin_amdgcn_readlane(a, 63), -pp[0][0]);
        pp[1][1] = wadd(__builtin_amdgcn_readlane(b, 63), -pp[0][1]);
      }
      // the king-move jobs' PSQT sums, on their slot lanes: the first four now, the rest (rare:
      // > 4 king-move children) four at a time
      int32_t jsum = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (jl[u] >= 0) { // (uniform)
          const int32_t s = wave_sum_dpp(jv[u]);
          if (lane == jl[u]) jsum = s;
        }
      }
      while (jrest) {
        int32_t v[4] = {0, 0, 0, 0};
        int vl[4] = {-1, -1, -1, -1};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (jrest) {
            const int l = __builtin_ctzll(jrest);
            jrest &= jrest - 1;
            int row, pos, cpc;
            job_rows(l, row, pos, cpc);
            v[u] = job_row_psqt(l, row), vl[u] = l;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int32_t s = wave_sum_dpp(v[u]);
          if (lane == vl[u]) jsum = s;
        }
      }
      int d0 = 0, d1 = 0;
      if (kinds == 15) {
        d0 = have ? 1 : pnd[0] >= 0 ? pnd[0] + 2 : P + 1 + (pst[0] ? 1 : 0);
        d1 = have ? 1 : pnd[1] >= 0 ? pnd[1] + 2 : P + 1 + (pst[1] ? 1 : 0);
      }
      else {
        if ((kinds & 3) == 1) d0 = n0 - (hit0 ? 1 : 0);
        if ((kinds >> 2) == 1) d1 = n1 - (hit1 ? 1 : 0);
      }
      const uint32_t c = (uint32_t)d0 | (uint32_t)d1 << 16;
      const uint32_t inc = scan_add(c); // (two 16-bit prefix sums; a pass's entries < 2^16)
      const uint32_t exc = inc - c, tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      const bool nx = q == nxpos;
      // ---- PSQT of the slot by side (a king-move perspective: its job's sum), slot metadata
      if (in && live) {
        int32_t sv[2] = {0, 0}; // the slot's PSQT at its bucket by side (0: the side to move)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int kd = hh ? kinds >> 2 : kinds & 3;
          int32_t v = 0;
          if (kd == 3) v = pp[hh][0];
          if (kd == 1) { // parent - from-row -+ the second row + the added rows
            const int32_t d1 = (hh ? s1 : s0) >= 2 ? -dq[hh][1] : dq[hh][1];
            v = wadd(pp[hh][bk == bp ? 0 : 1], wadd(wadd(-dq[hh][0], d1), wadd(dq[hh][2], dq[hh][3])));
          }
          v = kd == 2 ? jsum : v;
          *reinterpret_cast<int32_t *>(tf(tk0 + tix, offsetof(TileDesc, psq) + 8 * t + 4 * (hh != cst))) = v;
          sv[hh != cst] = v;
        }
        // the column-sliced stream's finish takes each evaluated position's PSQT value and
        // bucket from here (Network::evaluate's psqt term, a15 / a17), by output index
        if (pinfo && vld)
          pinfo[q == 0 ? (uint64_t)p : (uint64_t)np + off + (uint64_t)child_of(q)] =
              make_int2((int32_t)((uint32_t)sv[0] - (uint32_t)sv[1]) / 2, bk);
      }
      if (in) {
        *tf(tk0 + tix, offsetof(TileDesc, meta) + t) = (char)((live && vld ? 1 : 0) | bk << 1 | (q == 0 ? 16 : 0) | cst << 5);
        *reinterpret_cast<int16_t *>(tf(tk0 + tix, offsetof(TileDesc, adj) + 2 * t)) =
            (int16_t)(q == 0 ? 0 : child_of(q) - (q - 1));
      }
      if (live && q0 == 0) { // the parent loads the carry / cache rows: after their stores
        if (pnd[0] >= 0) pad_to(0, safe0);
        if (pnd[1] >= 0) pad_to(1, safe1);
      }
      // the parent's entries (the parent is lane 0: tile 0 of the pass, its delta region starts
      // at the cursor), before the jobs: a cache-row load is put while the lists' last scratch
      // stores are still the ones before it (put() checks the distance)
      if (live && q0 == 0 && lane == 0) {
        const uint32_t t0w = hs(tf0, stm != 0, xu, hu), t1w = hs(tf0, stm != 1, xu, hu);
        if (have) { // the parent is its predecessor's last child: pacc, one entry per list
          put(0, len0, LO_ZERO, M_SUB | HP | t0w | H_PAR_E | H_LAST);
          put(1, len1, LO_ZERO, M_SUB | HP | t1w | H_PAR_E | H_LAST);
        } else { // bias entry or the cache row; the rest follows (lane = square / row)
          put(0, len0, pnd[0] >= 0 ? lo_scr(2 + pkq[0]) : LO_BIAS, M_ADD | HZ | t0w | H_PAR_E);
          put(1, len1, pnd[1] >= 0 ? lo_scr(2 + 64 + pkq[1]) : LO_BIAS,
              M_ADD | HZ | t1w | H_PAR_E);
        }
      }
      if (live && q0 == 0 && !have) {
        const uint64_t lt2 = (1ull << lane) - 1;
#pragma unroll 1
        for (int hh = 0; hh < 2; ++hh) {
          const uint32_t tp = hs(tf0, stm != hh, xu, hu), b0 = (hh ? len1 : len0) + 1;
          const uint32_t kr = (uint32_t)(2 + 64 * hh + pkq[hh]); // the cache row (scratch row index)
          if (pnd[hh] >= 0) { // the cache row's differences: removed pieces, then added ones
            int spc;
            uint64_t bs, ba;
            cache_diff(64 * hh + pkq[hh], ppc, spc, bs, ba);
            if ((bs >> lane) & 1)
              put(hh, b0 + popcnt(bs & lt2), (uint32_t)feature_index(hh, lane, spc, pkq[hh]) * RS, M_SUB | tp | H_PAR_E);
            if ((ba >> lane) & 1)
              put(hh, b0 + popcnt(bs) + popcnt(ba & lt2), (uint32_t)feature_index(hh, lane, ppc, pkq[hh]) * RS,
                  M_ADD | tp | H_PAR_E);
            if (lane == 0) put(hh, b0 + pnd[hh], LO_ZERO, kr | tp | H_KST | H_LAST | H_PAR_E);
          } else {
            if (lane < P)
              put(hh, b0 + lane, ft_row(prow[hh][lane]) * RS, M_ADD | tp | H_PAR_E | (lane == P - 1 && !pst[hh] ? H_LAST : 0u));
            if (pst[hh] && lane == 0) put(hh, b0 + P, LO_ZERO, kr | tp | H_KST | H_LAST | H_PAR_E);
          }
          if (pnd[hh] >= 0 || pst[hh]) { // list hh stored the row: its snapshot and state
            uint32_t x = (uint32_t)ppc << (4 * (lane & 7));
            x = or8(x);
            const int kci = 64 * hh + pkq[hh];
            if ((lane & 7) == 0) ksnap[w][kci][lane >> 3] = x;
            kstate_set(hh, pkq[hh], 1 | hh << 1);
            uint32_t &sf = hh ? safe1 : safe0;
            sf = b0 + (uint32_t)(pnd[hh] >= 0 ? pnd[hh] : P) + GN_SCR_GAP; // the store's index + the gap
          }
        }
        ps::wave_sync();
      }
      rows += (tot & 0xFFFF) + (tot >> 16);
      pp_b += PP_T() - pp_t, pp_t = PP_T();
      // ---- tile by tile: reserve the tile's delta region, append its king-move jobs, close it
      // (the last tile of the pass stays open unless full).  ts0 / ts1: lane j = where tile j's
      // delta region starts in list 0 / 1.
      uint32_t ts0 = 0, ts1 = 0;
      auto excat = [&](int ln) -> uint32_t { // exclusive delta prefix at lane ln (n_in: the total)
        return ln >= n_in ? tot : (uint32_t)__builtin_amdgcn_readlane((int)exc, ln);
      };
      auto tile_lane0 = [&](int j) { return j == 0 ? 0 : c1 + 16 * (j - 1); };
      auto open_tile = [&](int j) {
        ts0 = lane == j ? len0 : ts0, ts1 = lane == j ? len1 : ts1;
        const uint32_t d = excat(j + 1 < ntp ? tile_lane0(j + 1) : n_in) - excat(tile_lane0(j));
        len0 += d & 0xFFFF, len1 += d >> 16;
      };
      auto close_tile = [&](int j) { // a tile the pass filled (or cut), not the pass's last
        const int fill = j == 0 ? tf0 + c1 : 16;
        if (lane >= fill && lane < 16) *tf(tk0 + j, offsetof(TileDesc, meta) + lane) = 0;
        const uint32_t pf = j == 0 ? p_first : p, tfi = j == 0 ? t_first : u_fill + (uint32_t)tile_lane0(j);
        if (lane == 0) *reinterpret_cast<uint4 *>(tf(tk0 + j, 0)) = make_uint4(len0, len1, pf, tfi);
      };
      int jc = 0;
      open_tile(0);
      // a job's slot descriptor in one register (one v_readlane per job): tile (< 8), side
      // refreshed, side to move, slot in tile, piece count, king destination, not castling
      const uint32_t jsq01 = ref1 ? w2 : w0, jsq23 = ref1 ? w3 : w1;
      const uint32_t jdesc = (uint32_t)tix | (uint32_t)ref1 << 3 | (uint32_t)cst << 4 | (uint32_t)t << 5 |
                             (uint32_t)cnt << 9 | ((jsq01 >> 16) & 63) << 15 | ((jsq23 & 0xFFFF) == 64 ? 1u << 21 : 0u);
      int ji = 0; // the job's index in the pass
      while (jm) {
        const int l = __builtin_ctzll(jm);
        jm &= jm - 1;
        const uint32_t jd = (uint32_t)__builtin_amdgcn_readlane((int)jdesc, l);
        const int jt = (int)(jd & 7), hh = (int)((jd >> 3) & 1), st = (int)((jd >> 4) & 1);
        const int tl = (int)((jd >> 5) & 15), cn = (int)((jd >> 9) & 63);
        while (jc < jt) close_tile(jc), ++jc, open_tile(jc);
        const bool nxl = q0 + l == nxpos;
        const int kt = (int)((jd >> 15) & 63);
        int row, pos, cpc;
        if (ji < 4) { // computed with the PSQT loads (LDS: no registers held across the pass)
          const uint32_t r = jrow_s[w][ji][lane];
          row = (int)(r & 0xFFFF) - 1, pos = (int)((r >> 16) & 0xFF), cpc = (int)(r >> 24);
        } else {
          const uint32_t sq01 = (uint32_t)__builtin_amdgcn_readlane((int)(hh ? w2 : w0), l),
                         sq23 = (uint32_t)__builtin_amdgcn_readlane((int)(hh ? w3 : w1), l);
          row = king_move_row_pc(ppc, hh, sq01 & 0xFFFF, kt, sq23 & 0xFFFF, sq23 >> 16, lane, pos, cpc);
        }
        ++ji;
        const uint32_t tw = hs(tl, hh != st, xu, hu);
        bool kuse = kc && ((jd >> 21) & 1); // not castling
        const int kci = 64 * hh + kt;
        const int kst = kuse ? kstate_of(hh, kt) : 0;
        // a cache row, once stored, stays with the list that stored it: the other list's
        // waves are not ordered with that list's stores inside a tile, so a second list
        // storing or loading the row could race with them
        const int own = (kst & 1) ? (kst >> 1) & 1 : -1;
        if (nxl && own >= 0 && own != hh) kuse = false; // the next parent's slot must be in list hh
        bool hit = false;
        uint64_t bs = 0, ba = 0;
        int spc = 0;
        if (kst & 1) {
          spc = (int)((ksnap[w][kci][lane >> 3] >> (4 * (lane & 7))) & 15);
          bs = __ballot(spc != cpc && spc != 0);
          ba = __ballot(spc != cpc && cpc != 0);
          const int nd = popcnt(bs) + popcnt(ba);
          hit = nd < cn && (!nxl || ((kst >> 1) & 1) == hh);
        }
        const int g = hit ? own : nxl ? hh : kuse && own >= 0 ? own : (len0 <= len1 ? 0 : 1);
        if (hit) pad_to(g, g ? safe1 : safe0); // the cache row load after the list's last scratch store
        const uint32_t base = g ? len1 : len0;
        const uint32_t L = H_LAST | (nxl ? H_PAR_E : 0u);
        const uint32_t kr = (uint32_t)(2 + kci); // the cache row (scratch row index)
        int ne;
        if (hit) {
          const int nd = popcnt(bs) + popcnt(ba);
          ne = nd + 2;
          const int ps = 1 + popcnt(bs & lt), pa = 1 + popcnt(bs) + popcnt(ba & lt);
          if (lane == 0) put(g, base, lo_scr(kr), M_ADD | HZ | tw);
          if ((bs >> lane) & 1) put(g, base + ps, (uint32_t)feature_index(hh, lane, spc, kt) * RS, M_SUB | tw);
          if ((ba >> lane) & 1) put(g, base + pa, (uint32_t)row * RS, M_ADD | tw);
          if (lane == 0) put(g, base + ne - 1, LO_ZERO, kr | tw | H_KST | L);
          rows += (uint32_t)(nd + 1);
        } else {
          ne = cn + 1 + (kuse ? 1 : 0);
          if (lane == 0) put(g, base, LO_BIAS, M_ADD | HZ | tw);
          if (row >= 0 && pos < cn) put(g, base + 1 + pos, (uint32_t)row * RS, M_ADD | tw | (!kuse && pos == cn - 1 ? L : 0u));
          if (kuse && lane == 0) put(g, base + ne - 1, LO_ZERO, kr | tw | H_KST | L);
          rows += (uint32_t)(cn + 1);
        }
        if (kuse) { // the cache row now holds this child's accumulator, stored by list g
          uint32_t x = (uint32_t)cpc << (4 * (lane & 7));
          x = or8(x);
          if ((lane & 7) == 0) ksnap[w][kci][lane >> 3] = x;
          kstate_set(hh, kt, 1 | g << 1);
          ps::wave_sync();
        }
        if (kuse) { // this slot's last entry stores to scratch
          uint32_t &sf = g ? safe1 : safe0;
          sf = base + (uint32_t)ne - 1 + GN_SCR_GAP;
        }
        if (g) len1 += (uint32_t)ne;
        else len0 += (uint32_t)ne;
      }
      while (jc < ntp - 1) close_tile(jc), ++jc, open_tile(jc);
      pp_d += PP_T() - pp_t, pp_t = PP_T();
      // ---- the delta entries of every lane, in its tile's reserved region
      {
        const uint32_t rel = exc - (uint32_t)__shfl((int)exc, tile_lane0(tix)); // (no borrow: prefix sums)
        const uint32_t at0 = (uint32_t)__shfl((int)ts0, tix) + (rel & 0xFFFF);
        const uint32_t at1 = (uint32_t)__shfl((int)ts1, tix) + (rel >> 16);
        const uint32_t t0w = hs(t, cst != 0, xu, hu), t1w = hs(t, cst != 1, xu, hu);
        if (in && live) {
          auto delta = [&](int g, uint32_t at, uint32_t lo2, uint32_t hi2, int s, int n, bool hit, uint32_t tw,
                           uint32_t L) {
            const uint32_t i0 = lo2 & 0xFFFF, i1 = lo2 >> 16, i2 = hi2 & 0xFFFF, i3 = hi2 >> 16;
            auto cl = [](uint32_t r) { return (r < (uint32_t)FT_INPUTS ? r : (uint32_t)FT_BIAS_ROW) * RS; };
            const uint32_t r1 = cl(s >= 2 ? i1 : i2), r2 = cl(s >= 2 ? i2 : i3), r3 = cl(i3);
            const uint32_t f1 = s >= 2 ? M_SUB : M_ADD;
            if (!hit) {
              put(g, at, cl(i0), M_SUB | HP | tw | (n == 1 ? L : 0u));
              if (n > 1) put(g, at + 1, r1, f1 | tw | (n == 2 ? L : 0u));
              if (n > 2) put(g, at + 2, r2, M_ADD | tw | (n == 3 ? L : 0u));
              if (n > 3) put(g, at + 3, r3, M_ADD | tw | L);
            } else { // the from-row is in the cached base
              put(g, at, r1, f1 | HB | tw | (n == 2 ? L : 0u));
              if (n > 2) put(g, at + 1, r2, M_ADD | tw | (n == 3 ? L : 0u));
              if (n > 3) put(g, at + 2, r3, M_ADD | tw | L);
            }
          };
          if ((kinds & 3) == 1) delta(0, at0, w0, w1, s0, n0, hit0, t0w, H_LAST | (nx ? H_PAR_E : 0u));
          if ((kinds >> 2) == 1) delta(1, at1, w2, w3, s1, n1, hit1, t1w, H_LAST | (nx ? H_PAR_E : 0u));
        }
      }
      // ---- the pass's last tile stays open
      uint32_t lbm = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b)
        if (__ballot(tix == ntp - 1 && ((mybit >> b) & 1))) lbm |= 1u << b;
      if (ntp > 1) p_first = p, t_first = u_fill + (uint32_t)tile_lane0(ntp - 1);
      tile_k = tk0 + (uint32_t)(ntp - 1);
      t_fill = ntp == 1 ? tf0 + n_in : n_in - tile_lane0(ntp - 1);
      tile_bm = ntp == 1 ? tile_bm | lbm : lbm;
      u_fill += (uint32_t)n_in;
      pp_c += PP_T() - pp_t;
      if (t_fill == 16) flush();
    }
  }
  if (t_fill) flush();
#ifdef GN_FAULT_PLAN_BLOCK
  // the first plan launch of the process reports an entry overflow for this block (err bit 0) and
  // leaves its last tile's list ends past the block's entry region, as round 4's plan bug did:
  // the stream must clamp them (elim) and stay inside the region, and the call must fail
  if (blk == (uint32_t)(GN_FAULT_PLAN_BLOCK) && tile_k > 0) {
    int armed = lane == 0 ? atomicExch(&gn_fault_armed, 0) : 0;
    if (__builtin_amdgcn_readfirstlane(armed)) {
      if (lane == 0) *reinterpret_cast<uint2 *>(tf(tile_k - 1, 0)) = make_uint2(rtot + 4096u, rtot + 4096u);
      bad |= 1u;
    }
  }
#endif
  if (lane == 0) btiles[blk] = tile_k;
  // error bits: 1 entries beyond the block's region (eoff under-counted), 4 a scratch-row load
  // closer than GN_SCR_GAP to its list's last scratch store; neither can happen by construction
  const uint32_t werr = __ballot(bad & 1u) ? 1u : 0u, werr4 = __ballot(bad & 4u) ? 4u : 0u;
  if (lane == 0) {
    if ((uint64_t)len0 + len1 > (uint64_t)(rtot - ENT_SPARE) || werr) atomicOr(err, 1u);
    if (werr4) atomicOr(err, 4u);
    if (rows_out) atomicAdd(rows_out, (unsigned long long)rows);
    if (pads_out && pads) atomicAdd(pads_out, (unsigned long long)pads);
    PP_ADD(0, pp_a), PP_ADD(1, pp_b), PP_ADD(2, pp_c), PP_ADD(3, pp_d);
    SP_ADD(6, pads), SP_ADD(7, fpads);
  }
  (void)pads, (void)fpads;
}

// ----------------------------------------------------------------- stream --
// SL > 1: the accumulator columns split over SL launches (slice = 0 .. SL - 1), each walking
// every entry of the plan over its own L1 / SL columns (pairs j, j + L1 / 2 of the transform
// together), so that an XCD's L2 holds the slice's rows of the king buckets in flight (the
// whole 3072-wide rows of one bucket pair, 8.6 MB, exceed its 4 MB).  A slice's fc_0 sums are
// partial: every slice stores them (part[slice][position][16], position = the output index:
// parent P, or np + child) and slice 0 the position's PSQT value and layer-stack bucket
// (pinfo[position]); slice_finish_kernel adds the SL sums (wrapping int32 adds, as the LDS
// atomics: the sum is the whole-row kernel's exactly) and runs the rest of the layer stack.
// (The last slice finishing in its own launch, one of its two waves per bucket, took 59.6 ms
// against 49 for the others.)
template <int L1, int SL = 1>
__global__ void __launch_bounds__(L1 / SL / 8) __attribute__((amdgpu_waves_per_eu(SL > 1 ? GN_SLICE_WPE : GN_EXPAND_WPE)))
    stream_eval_kernel(NetDevice net, const uint64_t *__restrict__ offsets, uint32_t np, uint32_t K, uint32_t b0,
                       uint32_t b1, int swz,
                       const uint64_t *__restrict__ eoff, const uint64_t *__restrict__ ent,
                       const TileDesc *__restrict__ tiles, const uint32_t *__restrict__ btiles,
                       const uint32_t *__restrict__ order, int2 *__restrict__ out_parent, int2 *__restrict__ out_child,
                       uint32_t *__restrict__ pool, int use_scr, uint32_t *__restrict__ err,
                       uint32_t *__restrict__ claim, int slice, int32_t *__restrict__ part, uint64_t npos,
                       int2 *__restrict__ pinfo) {
  using namespace ps;
  constexpr int LC = L1 / SL; // this launch's columns
  constexpr int G = LC / 16;  // threads per perspective group (whole waves)
  constexpr int NT = 2 * G, NW = NT / 64, TILE = 16, XS = tile_xs(L1, SL), KS = LC / 64,
                KPW = KS / NW;
  constexpr int KSF = L1 / 64; // fc_0 k-steps of the whole net
  constexpr uint32_t RS = ft_row_stride(L1);
  static_assert(G % 64 == 0 && KS % NW == 0 && KPW % 2 == 0 && L1 % SL == 0, "geometry");
  // the slice's first column pair in bytes (its low columns; the high ones L1 bytes further)
  const uint32_t cofs = SL > 1 ? (uint32_t)slice * (uint32_t)LC : 0u;
  __shared__ __attribute__((aligned(16))) uint8_t xt[TILE * XS];
  // fc_0 partial sums [position][output], rows padded to 20 dwords: the 4 lane groups of an
  // atomic (kg) then fall on different banks (a 16-dword row put all 4 on the same bank)
  constexpr int AS = 20;
  __shared__ __attribute__((aligned(16))) int32_t acc0[2][16 * AS];
  __shared__ __attribute__((aligned(16))) uint8_t in1[2][TILE][32];
  __shared__ int32_t fwd[2][TILE];
  __shared__ uint32_t sslot, sblk;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hu = __builtin_amdgcn_readfirstlane((tid / G) & 1);
  for (int i = tid; i < 2 * 16 * AS; i += NT) (&acc0[0][0])[i] = 0;
  // this launch evaluates blocks [b0, b1).  swz: XCD x (= dispatch index mod 8) takes the x-th
  // contiguous eighth of them; otherwise (default) every workgroup claims the next block of the
  // order with one atomic (claim[0], zeroed per launch), so blocks are taken in order wherever
  // a workgroup slot frees up: XCDs that run faster take more blocks (measured: the even XCDs
  // of an MI355X finish the static split 2-3 % after the odd ones), and the resident blocks of
  // every XCD stay neighbours in the king order
  // The grid has nblk + nblk / 16 + 8 workgroups then: the hardware hands every XCD the same
  // number of them, so a faster XCD needs spare workgroups to take more blocks, and the ones
  // left over once every block is claimed end here.
  // swz 2: each XCD claims the blocks of its own contiguous eighth of the order (claim[x]), so
  // that the blocks resident on one XCD (sharing its L2) are neighbours in the king order, and
  // one that has run out takes the next unclaimed block of another XCD's eighth.
  const uint32_t nblk = b1 - b0;
  const uint32_t vgrid = swz == 1 ? 8 * ((nblk + 7) / 8) : nblk;
  uint32_t v = blockIdx.x;
  if (swz == 0) {
    if (tid == 0) sblk = atomicAdd(claim, 1u);
    __syncthreads();
    v = sblk;
  } else if (swz == 2) {
    if (tid == 0) {
      uint32_t x;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
      x &= 7;
      const uint32_t per = (nblk + 7) / 8;
      uint32_t got = ~0u;
      for (uint32_t t = 0; t < 8 && got == ~0u; ++t) {
        const uint32_t y = (x + t) & 7, lo = y * per, hi = lo + per < nblk ? lo + per : nblk;
        if (lo >= hi || __hip_atomic_load(claim + y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= hi - lo) continue;
        const uint32_t i = atomicAdd(claim + y, 1u);
        if (i < hi - lo) got = lo + i;
      }
      sblk = got;
    }
    __syncthreads();
    v = sblk; // ~0u: every block is claimed (v >= vgrid below)
  }
  if (v >= vgrid) return;
  uint32_t blk = v;
  if (swz == 1) {
    const uint32_t b8 = (nblk + 7) / 8;
    blk = (v & 7) * b8 + (v >> 3);
    if (blk >= nblk) return;
  }
  blk = order ? order[b0 + blk] : blk + b0; // order: a permutation of the blocks (block_order)
  const uint32_t pbeg = blk * K, pend = pbeg + K < np ? pbeg + K : np;
  const uint64_t us_b = pbeg + offsets[pbeg];
  const uint32_t ntiles = btiles[blk];
  const TileDesc *T = tiles + us_b / 16 + (uint64_t)(K + 2) * blk; // as plan_kernel
  const uint64_t rbeg = eoff[pbeg] + (uint64_t)ENT_SPARE * blk, rend = eoff[pend] + (uint64_t)ENT_SPARE * (blk + 1);
  // a list never ends past the block's entry bound (the region less its ENT_SPARE entries): a
  // tile end beyond it can only come from a plan that overflowed, which the plan reports (err
  // bit 0, the call fails); clamped, the entry loads (and their prefetch, 8 ahead) stay inside
  // the region whatever the descriptors say
  const uint32_t elim = (uint32_t)(rend - rbeg) - ENT_SPARE;
#ifdef GN_XCD_PROF
  const unsigned long long xp_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- scratch slot (carry + king-cache rows) from this XCD's pool: never waits on another
  // workgroup; the pool (POOL_PER_XCD slots) outnumbers the workgroups an XCD holds
  uint32_t scr = 0, my_slot = 0;
  if (use_scr) {
    if (tid == 0) {
      uint32_t x;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
      x &= 7;
      uint32_t *wd = pool + 8 * x;
      int got = -1;
      for (int it = 0; it < 4096 && got < 0; ++it) {
        const int wi = (int)((it + (v >> 3)) & 7);
        uint32_t cur = __hip_atomic_load(wd + wi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (cur != 0xFFFFFFFFu) {
          const int bit = __builtin_ctz(~cur);
          const uint32_t old = __hip_atomic_fetch_or(wd + wi, 1u << bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (!(old & (1u << bit))) {
            got = (int)(x * POOL_PER_XCD + 32 * wi + bit);
            break;
          }
          cur = old | (1u << bit);
        }
        if (got < 0 && wi == 7) __builtin_amdgcn_s_sleep(4);
      }
      if (got < 0) atomicOr(err, 2u), got = 0; // cannot happen (pool > resident workgroups); reported
      sslot = (uint32_t)got;
    }
    __syncthreads();
    my_slot = sslot;
    scr = (uint32_t)FT_ROWS + (uint32_t)SCR_ROWS * my_slot;
  }

  // the stream and the tile loop are compiled once per perspective group (HU = hu): the
  // list's direction and the group's carry row are then constants of the code
  auto run_group = [&](auto hu_c) {
  constexpr int HU = decltype(hu_c)::value;
  // ---- per-thread stream state: ONE continuous pipeline per group over the block's list.
  // Entries arrive through scalar loads (their own counter, lgkmcnt), 4 at a time and two
  // groups of 4 ahead, so waiting for an entry never waits for the row loads in flight;
  // rows are loaded one group of 4 ahead of consumption, also across tile boundaries
  // (the next tile's first rows are in flight during this tile's layer stack).
  // the accumulator (A), the parent accumulator (PA) and the sibling base (BA) of this lane's 16
  // columns as 8 dwords each (the low half's 8 columns, then the high half's)
  uint32_t PA[8] = {0, 0, 0, 0, 0, 0, 0, 0}, BA[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  constexpr int RD = SL > 1 ? GN_SLICE_RING : GN_RING;
  static_assert(RD == 4 || RD == 5 || RD == 6 || RD == 8, "ring depth");
  // the ring's waits: before an entry is consumed, its two loads are older than the RD - 1 later
  // entries' (2 loads each); the layer stack waits for every load older than the ring's RD entries
  constexpr int RWAIT = 2 * (RD - 1), RWAIT_PV = 2 * RD;
  // entries per scalar group load: 4 (s_load_dwordx8) or 8 (x16; rings of 5 or 6 use the first RD)
  constexpr int GV = RD;
  ushort8 rlo[RD], rhi[RD];
  uint32_t eh[RD]; // hi words of the entries in flight
  uint32_t bq = 0; // buckets done (acc0 / in1 / fwd buffer parity)
  // SL > 1: this wave's fc_0 weights of one bucket (its 8 k-steps of the slice, in the MFMA's
  // operand order) stay in registers across tiles (a game's bucket changes rarely); a tile whose
  // first bucket is not the cached one loads it at the tile's start, so that the loads are older
  // than the ring's row loads of the tile's last entries and the layer stack waits for them alone
  // (vmcnt counts in issue order: loads issued at the layer stack wait behind the ring's 8)
  int4v wc[8]; // (no initial value: read only after a fill)
  int cb = 8; // the cached bucket (8: none)
  const __amdgpu_buffer_rsrc_t w0r = __builtin_amdgcn_make_buffer_rsrc(
      (void *)net.w0f, 0, (int)((size_t)PSQT_BUCKETS * KSF * 1024), 0x00020000);
  const uint32_t wl16 = (uint32_t)(threadIdx.x & 63) * 16;
  // the 8 k-steps of bucket b for this wave (side = the wave's perspective group, the slice's
  // k-steps of that side): invisible to the compiler's waits like the ring (wc_wait below)
  auto wc_load = [&](int b) {
    const uint32_t so = ((uint32_t)b * KSF + (uint32_t)(24 * HU + 8 * slice)) * 1024u;
    asm volatile("buffer_load_dwordx4 %0, %8, %9, %10 offen\n\t"
                 "buffer_load_dwordx4 %1, %8, %9, %10 offen offset:1024\n\t"
                 "buffer_load_dwordx4 %2, %8, %9, %10 offen offset:2048\n\t"
                 "buffer_load_dwordx4 %3, %8, %9, %10 offen offset:3072\n\t"
                 "buffer_load_dwordx4 %4, %8, %9, %11 offen\n\t"
                 "buffer_load_dwordx4 %5, %8, %9, %11 offen offset:1024\n\t"
                 "buffer_load_dwordx4 %6, %8, %9, %11 offen offset:2048\n\t"
                 "buffer_load_dwordx4 %7, %8, %9, %11 offen offset:3072"
                 : "+v"(wc[0]), "+v"(wc[1]), "+v"(wc[2]), "+v"(wc[3]), "+v"(wc[4]), "+v"(wc[5]), "+v"(wc[6]),
                   "+v"(wc[7]) // ("+v": the fill overwrites the cache's own registers, no copies)
                 : "v"(wl16), "s"(w0r), "s"(so), "s"(so + 4096u));
  };
  // wait for the cache's loads: vmcnt(8) when at least 8 vector-memory operations were issued
  // after them (the ring's loads of the tile's last 4 entries: in-order completion), else all
#define GN_WC_WAIT(N) asm volatile("s_waitcnt vmcnt(%8)" : "+v"(wc[0]), "+v"(wc[1]), "+v"(wc[2]), "+v"(wc[3]), \
                                   "+v"(wc[4]), "+v"(wc[5]), "+v"(wc[6]), "+v"(wc[7]) : "n"(N))
  typedef uint32_t u8e __attribute__((ext_vector_type(2 * GV), aligned(8)));
  typedef const __attribute__((address_space(4))) u8e cu8e;
  typedef const __attribute__((address_space(4))) uint64_t cu64;
  cu64 *EL = (cu64 *)(HU ? ent + rend : ent + rbeg);
  // entries i .. i + GV - 1 of this group's list by one s_load_dwordx8 / x16 (list 1 is stored
  // downward: its entries arrive reversed, see elo / ehi)
  auto group = [&](uint32_t i) -> u8e { return *(cu8e *)(HU ? EL - GV - i : EL + i); };
  auto elo = [&](const u8e v, int r) -> uint32_t { return HU ? v[2 * (GV - 1 - r)] : v[2 * r]; };
  auto ehi = [&](const u8e v, int r) -> uint32_t { return HU ? v[2 * (GV - 1 - r) + 1] : v[2 * r + 1]; };
  int tl0 = tid;
  asm volatile("" : "+v"(tl0));
  const int jt = tl0 % G;
  const uint32_t j16 = 16 * jt + cofs;
  typedef int sq4 __attribute__((ext_vector_type(4)));
  const uint64_t ftp = (uint64_t)(uintptr_t)net.ft;
  const sq4 rsq = {__builtin_amdgcn_readfirstlane((int)(uint32_t)ftp),
                   __builtin_amdgcn_readfirstlane((int)(uint32_t)(ftp >> 32) & 0xFFFF),
                   (int)(((size_t)ZERO_ROW + 1) * RS), 0x00020000};
  // this slot's rows from the first scratch row, less the SCR bit the entry carries in lo
  const uint32_t scr_off = (scr - (uint32_t)FT_ROWS) * RS - L_SCR;
  auto offset = [&](uint32_t lo, uint32_t h) -> uint32_t {
    (void)h;
#ifdef GN_ABLATE_ROWS
    (void)lo, (void)h;
    return (uint32_t)FT_BIAS_ROW * RS; // timing diagnostics build only: every row from L1 / L2
#else
    return lo + ((uint32_t)((int32_t)lo >> 31) & scr_off);
#endif
  };
  auto issue = [&](int r, uint32_t lo, uint32_t h) {
    eh[r] = h;
    // the ring's loads are invisible to the compiler's wait insertion (which, merging the
    // paths of the entry kinds at the loop head, waits for far more of the ring than an entry
    // needs); consume() waits for exactly its own row: see ring_wait
#ifndef GN_ROW_POLICY
#define GN_ROW_POLICY "" // A/B: cache-policy modifiers of the row loads (e.g. " nt")
#endif
    asm volatile("buffer_load_dwordx4 %0, %2, %3, %4 offen" GN_ROW_POLICY "\n\t"
                 "buffer_load_dwordx4 %1, %2, %3, %4 offen offset:%5" GN_ROW_POLICY
                 : "=&v"(rlo[r]), "=&v"(rhi[r])
                 : "v"(j16), "s"(rsq), "s"(offset(lo, h)), "n"(L1));
  };
  // before entry r is consumed: its two loads are the oldest of the 8 in flight (the 3 later
  // entries of the last revolution and the earlier ones of this one were issued since); any
  // other memory operation in between (a drained store, the layer stack's loads) only makes
  // vmcnt(6) wait for more.  The "+v" ties the row registers to the wait: no use before it.
  // (one wait form only: a second form behind a branch made the compiler copy ring registers
  // before their wait at the join -- tests/test_host.py::test_ring_registers_untouched_in_flight.
  // A weight-cache fill at a tile's start is younger than the RD entries then in flight, so the
  // next waits also wait for its loads: once per bucket change)
  auto ring_wait = [&](int r) {
    asm volatile("s_waitcnt vmcnt(%2)" : "+v"(rlo[r]), "+v"(rhi[r]) : "n"(RWAIT));
  };
  uint32_t A[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto consume = [&](int r) {
    ring_wait(r);
    const uint32_t h = eh[r];
#ifdef GN_AB_SALU_PLUS // timing diagnostics only: N extra independent scalar ALU instructions per entry
    {
      uint32_t d0, d1;
      asm volatile(".rept " GN_STR(GN_AB_SALU_PLUS) " / 2\n\ts_add_u32 %0, %2, 1\n\ts_add_u32 %1, %2, 2\n\t.endr"
                   : "=&s"(d0), "=&s"(d1) : "s"(h));
    }
#endif
#ifdef GN_AB_VALU_PLUS // timing diagnostics only: N extra independent vector ALU instructions per entry
    {
      uint32_t d0, d1;
      asm volatile(".rept " GN_STR(GN_AB_VALU_PLUS) " / 2\n\tv_mov_b32 %0, %2\n\tv_mov_b32 %1, %2\n\t.endr"
                   : "=&v"(d0), "=&v"(d1) : "v"(j16));
    }
#endif
    // every entry is one 16-bit multiply-add per dword, acc = src + sg * row, its multiplier
    // sg (1, 0xFFFF = -1, 0) the low half of h as the instruction's scalar operand; src is
    // the accumulator, or (an init) 0 / the parent / the sibling base at a slot's first entry
    // (wrapping int16, as the accumulators).  The decode is a branch tree on h's init field, one
    // test per branch, each kind with its own multiply-adds (the compiler's version of this tree
    // copied the source registers on every path and spilled): a plain entry costs two scalar
    // instructions, an init five to seven.
#ifdef GN_AB_WHOLE_CDECODE // diagnostics: the whole-row stream with the compiler's decode (round 5's)
    if constexpr (SL == 1) {
      const unsigned short sg = (unsigned short)h;
      const uint32_t init = (h >> 16) & 3u;
      ushort8 lo = __builtin_bit_cast(ushort8, make_uint4(A[0], A[1], A[2], A[3]));
      ushort8 hi = __builtin_bit_cast(ushort8, make_uint4(A[4], A[5], A[6], A[7]));
      if (init) {
        asm volatile("");
        if (init == 2) {
          lo = __builtin_bit_cast(ushort8, make_uint4(PA[0], PA[1], PA[2], PA[3]));
          hi = __builtin_bit_cast(ushort8, make_uint4(PA[4], PA[5], PA[6], PA[7]));
        } else if (init == 3) {
          lo = __builtin_bit_cast(ushort8, make_uint4(BA[0], BA[1], BA[2], BA[3]));
          hi = __builtin_bit_cast(ushort8, make_uint4(BA[4], BA[5], BA[6], BA[7]));
        } else {
          lo = ushort8{}, hi = ushort8{};
        }
      }
      lo = rlo[r] * sg + lo, hi = rhi[r] * sg + hi;
      const uint4 l4 = __builtin_bit_cast(uint4, lo), h4 = __builtin_bit_cast(uint4, hi);
      A[0] = l4.x, A[1] = l4.y, A[2] = l4.z, A[3] = l4.w, A[4] = h4.x, A[5] = h4.y, A[6] = h4.z, A[7] = h4.w;
      if (init == 2) {
        asm volatile("");
#pragma unroll
        for (int i = 0; i < 8; ++i) BA[i] = A[i];
      }
    } else
#endif
    {
      const uint4 rl = __builtin_bit_cast(uint4, rlo[r]), rh = __builtin_bit_cast(uint4, rhi[r]);
      uint32_t t;
#define GN_MAD8(SRC)                                                                                        \
  "v_pk_mad_u16 %[a0], %[r0], %[h], %[" SRC "0] op_sel_hi:[1,0,1]\n\t"                                       \
  "v_pk_mad_u16 %[a1], %[r1], %[h], %[" SRC "1] op_sel_hi:[1,0,1]\n\t"                                       \
  "v_pk_mad_u16 %[a2], %[r2], %[h], %[" SRC "2] op_sel_hi:[1,0,1]\n\t"                                       \
  "v_pk_mad_u16 %[a3], %[r3], %[h], %[" SRC "3] op_sel_hi:[1,0,1]\n\t"                                       \
  "v_pk_mad_u16 %[a4], %[r4], %[h], %[" SRC "4] op_sel_hi:[1,0,1]\n\t"                                       \
  "v_pk_mad_u16 %[a5], %[r5], %[h], %[" SRC "5] op_sel_hi:[1,0,1]\n\t"                                       \
  "v_pk_mad_u16 %[a6], %[r6], %[h], %[" SRC "6] op_sel_hi:[1,0,1]\n\t"                                       \
  "v_pk_mad_u16 %[a7], %[r7], %[h], %[" SRC "7] op_sel_hi:[1,0,1]\n\t"
      asm volatile("s_and_b32 %[t], %[h], 0x30000\n\t"
                   "s_cbranch_scc0 .Lgn_plain%=\n\t"
                   "s_bitcmp1_b32 %[h], 17\n\t"
                   "s_cbranch_scc0 .Lgn_zero%=\n\t"
                   "s_bitcmp1_b32 %[h], 16\n\t"
                   "s_cbranch_scc0 .Lgn_pacc%=\n\t"
                   GN_MAD8("b")
                   "s_branch .Lgn_end%=\n"
                   ".Lgn_pacc%=:\n\t"
                   GN_MAD8("p")
                   "v_mov_b32 %[b0], %[a0]\n\t"
                   "v_mov_b32 %[b1], %[a1]\n\t"
                   "v_mov_b32 %[b2], %[a2]\n\t"
                   "v_mov_b32 %[b3], %[a3]\n\t"
                   "v_mov_b32 %[b4], %[a4]\n\t"
                   "v_mov_b32 %[b5], %[a5]\n\t"
                   "v_mov_b32 %[b6], %[a6]\n\t"
                   "v_mov_b32 %[b7], %[a7]\n\t"
                   "s_branch .Lgn_end%=\n"
                   ".Lgn_zero%=:\n\t"
                   "v_pk_mul_lo_u16 %[a0], %[r0], %[h] op_sel_hi:[1,0]\n\t"
                   "v_pk_mul_lo_u16 %[a1], %[r1], %[h] op_sel_hi:[1,0]\n\t"
                   "v_pk_mul_lo_u16 %[a2], %[r2], %[h] op_sel_hi:[1,0]\n\t"
                   "v_pk_mul_lo_u16 %[a3], %[r3], %[h] op_sel_hi:[1,0]\n\t"
                   "v_pk_mul_lo_u16 %[a4], %[r4], %[h] op_sel_hi:[1,0]\n\t"
                   "v_pk_mul_lo_u16 %[a5], %[r5], %[h] op_sel_hi:[1,0]\n\t"
                   "v_pk_mul_lo_u16 %[a6], %[r6], %[h] op_sel_hi:[1,0]\n\t"
                   "v_pk_mul_lo_u16 %[a7], %[r7], %[h] op_sel_hi:[1,0]\n\t"
                   "s_branch .Lgn_end%=\n"
                   ".Lgn_plain%=:\n\t"
                   GN_MAD8("a")
                   ".Lgn_end%=:"
                   // (early clobbers: the tree writes a0 .. while it still reads the later inputs, so
                   // no input may share a register with an output -- without "&" the compiler may
                   // give an output and an input of equal value one register)
                   : [a0] "+&v"(A[0]), [a1] "+&v"(A[1]), [a2] "+&v"(A[2]), [a3] "+&v"(A[3]), [a4] "+&v"(A[4]),
                     [a5] "+&v"(A[5]), [a6] "+&v"(A[6]), [a7] "+&v"(A[7]), [b0] "+&v"(BA[0]), [b1] "+&v"(BA[1]),
                     [b2] "+&v"(BA[2]), [b3] "+&v"(BA[3]), [b4] "+&v"(BA[4]), [b5] "+&v"(BA[5]), [b6] "+&v"(BA[6]),
                     [b7] "+&v"(BA[7]), [t] "=&s"(t)
                   : [h] "s"(h), [p0] "v"(PA[0]), [p1] "v"(PA[1]), [p2] "v"(PA[2]), [p3] "v"(PA[3]),
                     [p4] "v"(PA[4]), [p5] "v"(PA[5]), [p6] "v"(PA[6]), [p7] "v"(PA[7]), [r0] "v"(rl.x),
                     [r1] "v"(rl.y), [r2] "v"(rl.z), [r3] "v"(rl.w), [r4] "v"(rh.x), [r5] "v"(rh.y),
                     [r6] "v"(rh.z), [r7] "v"(rh.w)
                   : "scc");
#undef GN_MAD8
    }
    if (h & H_LAST) {
      const ushort8 lo = __builtin_bit_cast(ushort8, make_uint4(A[0], A[1], A[2], A[3]));
      const ushort8 hi = __builtin_bit_cast(ushort8, make_uint4(A[4], A[5], A[6], A[7]));
      // the slot's LDS offset: a shift of hi (slot * XS + side * LC / 2 in 16-B units), or for the
      // whole-row 3072 stream slot * 2 + side
      constexpr bool FIELD16 = lds_field16(XS, LC);
      const uint32_t la = FIELD16 ? (h >> H_LDS_SH) << 4
                                  : (h >> (H_LDS_SH + 1)) * (uint32_t)XS + ((h >> H_LDS_SH) & 1) * (uint32_t)(LC / 2);
#ifdef GN_AB_NO_TRANSFORM // timing diagnostics only (wrong results): the accumulator's low bytes, untransformed
      *reinterpret_cast<uint2 *>(xt + la + 8 * jt) = make_uint2(lo[0] | (uint32_t)hi[0] << 16, lo[1]);
#else
      *reinterpret_cast<uint2 *>(xt + la + 8 * jt) = transform8(lo, hi);
#endif
      if (h & H_X) {
      if (h & (H_PAR_E & ~H_X)) {
        asm volatile("");
#pragma unroll
        for (int i = 0; i < 8; ++i) PA[i] = A[i];
      }
      if (h & (H_KST & ~H_X)) { // the accumulator to its king-cache row
        asm volatile("");
        const uint32_t so = (scr + (h & 0xFFFFu)) * RS;
#ifndef GN_KC_ASM_POLICY
// cache policy of the king-cache stores: "" = default.  The same-address store -> load order
// the reload relies on is pinned for default-policy stores only (kernels.h); non-temporal
// (" nt") measured 205.5 -> 205.0 ms, within noise, so it stays an A/B build option
#define GN_KC_ASM_POLICY ""
#endif
        // Both halves in one asm block: the high half at the instruction's immediate offset, and a
        // wait state after the pair before any VALU may overwrite their data registers.  (As two
        // builtins, the whole-row kernel at its 96-VGPR cap computed the second address into a data
        // register of the first store in the very next instruction -- `buffer_store_dwordx4
        // v[2:5] ...; v_add_u32 v4, 0xc00, v1` -- with no wait state between: the king-cache rows
        // then held wrong values now and then, round 6, test_stream_column_slices_equal_whole_rows.
        // A VALU write to the data VGPRs of a > 64-bit store needs one wait state on this family.)
        static_assert(L1 < 4096, "the high half's offset fits the 12-bit immediate");
        asm volatile("buffer_store_dwordx4 %0, %2, %3, %4 offen" GN_KC_ASM_POLICY "\n\t"
                     "buffer_store_dwordx4 %1, %2, %3, %4 offen offset:%5" GN_KC_ASM_POLICY "\n\t"
                     "s_nop 0"
                     :
                     : "v"(__builtin_bit_cast(int4v, lo)), "v"(__builtin_bit_cast(int4v, hi)), "v"(j16), "s"(rsq),
                       "s"(so), "n"(L1)
                     : "memory");
        // no drain: the ring's vmcnt(6) still covers an entry's own loads with these two stores
        // outstanding (loads complete in order, so >= 2 of the >= 4 completions it waits for are
        // that entry's loads), and a later load of the row is issued after the store in program
        // order by the same lanes (the plan keeps it >= 4 entries behind)
      }
      }
    }
  };
  uint32_t pos = 0; // the next entry to consume: entries pos .. pos + 3 have their rows in flight
  u8e gp = group(RD); // the entries whose rows the next revolution issues (prefetched)
  u8e gw;            // ... and this revolution's
  {
    const u8e g0 = group(0);
#pragma unroll
    for (int r = 0; r < RD; ++r) issue(r, elo(g0, r), ehi(g0, r));
  }

  // tile slot sl's adj value (TileDesc.adj, the chained walk's output reorder) for a lane-varying
  // slot: the 8 words by scalar loads (no vector load: it would make the compiler wait for the
  // ring's loads in flight), into lanes 0..7 of one register, each lane fetching its word by
  // ds_bpermute (an 8-way select would keep 7 lane masks in SGPRs: spills)
  auto adj_of = [&](const TileDesc *Dt, int sl) -> int {
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    const cu32 *aw = (const cu32 *)reinterpret_cast<const uint32_t *>(Dt->adj);
    int vx = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(vx) : "s"((int)aw[i]), "i"(i));
    const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((sl >> 1) << 2, vx);
    return (int)(int16_t)(w >> (16 * (sl & 1)));
  };
  unsigned long long sp_s = 0, sp_w = 0, sp_l = 0, sp_m = 0, sp_n = 0;
  uint32_t sp_e0 = 0, sp_e1 = 0;
#pragma unroll 1
  for (uint32_t k = 0; k < ntiles; ++k) {
    const TileDesc *D = T + k;
    const unsigned long long t0 = SP_T();
#ifdef GN_STREAM_PROF
    if (wave == 0) {
      const uint32_t a0 = D->e_end[0], a1 = D->e_end[1];
      sp_m += (a0 - sp_e0) > (a1 - sp_e1) ? (a0 - sp_e0) : (a1 - sp_e1), sp_n += a0 - sp_e0 + a1 - sp_e1;
      sp_e0 = a0, sp_e1 = a1;
    }
#endif
    const uint32_t e_end = min((uint32_t)__builtin_amdgcn_readfirstlane(D->e_end[HU]), elim);
    const uint32_t p_first = __builtin_amdgcn_readfirstlane(D->p_first);
    const uint32_t first = __builtin_amdgcn_readfirstlane(D->first);
    uint32_t mw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      mw[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)reinterpret_cast<const uint32_t *>(D->meta)[i]);
    uint32_t bm = 0, pm = 0; // the tile's buckets, its parent slots
#pragma unroll
    for (int sl = 0; sl < TILE; ++sl) {
      const uint32_t m = (mw[sl >> 2] >> (8 * (sl & 3))) & 0xFF;
      if (m & 1) bm |= 1u << ((m >> 1) & 7);
      if (m & 16) pm |= 1u << sl;
    }
#ifdef GN_AB_NO_LS // timing diagnostics only (no outputs): the stream without its layer stack
    bm = 0;
#endif
    bool wpend = false; // (SL > 1) the cache was loaded at this tile's start
    const uint32_t pos0 = pos;
    if constexpr (SL > 1 && GN_WCACHE) {
      if (bm && !((bm >> cb) & 1)) {
        cb = __builtin_ctz(bm);
        wc_load(cb);
        wpend = true;
      }
    }
    // (SL > 1, slice > 0, in-place partial sums) this lane's 16 B of the previous slices' sums:
    // position wp of the tile, outputs 4 wj .. 4 wj + 3 (the writer's lane layout below); an
    // unevaluated slot reads position 0 (ignored).  Unconditional asm, waited with the cache
    // (no path join between the load and its wait)
    int4v pv;
    if constexpr (SL > 1 && GN_PART_N == 1) {
      const int ln = tid & 63, wp = ln >> 2, wj = ln & 3;
      const int adjv = adj_of(D, wp);
      const uint32_t m = (mw[wp >> 2] >> (8 * (wp & 3))) & 0xFF;
      const uint32_t P = p_first + (uint32_t)__builtin_popcount(pm & ((2u << wp) - 1)) - (pm & 1);
      const uint64_t q = !(m & 1) ? 0ull : ((pm >> wp) & 1) ? (uint64_t)P : (uint64_t)np + (us_b + first + wp - P - 1 + adjv);
      const int32_t *src = part + q * 16 + 4 * wj;
      if (slice > 0) asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(pv) : "v"(src));
    }
    // ---- the row stream of this group's list segment [pos, e_end): ring slot r holds entry i
    // with i % 4 == r, so a tile may begin and end anywhere in a revolution of 4 entries (a
    // revolution starts at a multiple of 4: it waits for its prefetched group of entries,
    // whose rows it issues, and prefetches the next); the steps of a partial revolution are
    // guarded by uniform tests, whole revolutions run unguarded (sliced stream)
#ifdef GN_AB_GUARDED // A/B (round 4): every entry behind its own guard
    constexpr bool REV = false;
#else
    constexpr bool REV = SL > 1; // (the whole-row stream, at its 96-VGPR cap, spills with it)
#endif
    // the tile's first partial revolution (guarded), then whole revolutions without per-entry
    // guards (each took 7 scalar instructions and a branch), then the last partial one (guarded)
    if constexpr (REV) {
      {
        const uint32_t r0 = pos % RD;
        if (r0 != 0) {
#pragma unroll
          for (int r = 1; r < RD; ++r)
            if (r0 <= (uint32_t)r && pos < e_end) consume(r), issue(r, elo(gw, r), ehi(gw, r)), ++pos;
        }
      }
#pragma unroll 1
      while (pos + RD <= e_end) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        gw = gp;
        gp = group(pos + 2 * RD);
#pragma unroll
        for (int r = 0; r < RD; ++r) consume(r), issue(r, elo(gw, r), ehi(gw, r));
        pos += RD;
      }
      if (pos < e_end) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        gw = gp;
        gp = group(pos + 2 * RD);
        consume(0), issue(0, elo(gw, 0), ehi(gw, 0));
        ++pos;
#pragma unroll
        for (int r = 1; r < RD - 1; ++r)
          if (pos < e_end) consume(r), issue(r, elo(gw, r), ehi(gw, r)), ++pos;
      }
    } else {
#pragma unroll 1
      while (pos < e_end) {
        const uint32_t r0 = pos % RD;
        if (r0 == 0) {
          // scalar loads complete out of order, so any use waits for all of them: wait once
          // here (lgkmcnt(0): the prefetch of the previous revolution), take this revolution's
          // entries, and only then prefetch the next group, which nothing uses before the next
          __builtin_amdgcn_s_waitcnt(0xC07F);
          gw = gp;
          gp = group(pos + 2 * RD);
          consume(0), issue(0, elo(gw, 0), ehi(gw, 0));
          ++pos;
        }
#pragma unroll
        for (int r = 1; r < RD; ++r)
          if (r0 <= (uint32_t)r && pos < e_end) consume(r), issue(r, elo(gw, r), ehi(gw, r)), ++pos;
      }
    }
    asm volatile("" ::: "memory");
    const unsigned long long t1 = SP_T();
#ifndef GN_AB_NO_BARRIER // timing diagnostics only (racy, wrong results): the layer stack without barriers
    __syncthreads();
#endif
    const unsigned long long t2 = SP_T();
    sp_s += t1 - t0, sp_w += t2 - t1;
    // ---- layer stack: per bucket of the tile, fc_0 by all waves (int8 MFMA over this wave's
    // k-steps, partial sums by LDS integer atomics, exact), then one wave finishes it
    const uint64_t u0 = us_b + first;
    if constexpr (SL > 1) {
      // the cache's loads (issued before the tile's entries) are complete once at most the 8
      // youngest operations are outstanding: the ring's loads of this list's last RD entries,
      // when the tile had RD entries or more since the fill; otherwise wait for everything.
      // The tied wait is unconditional (no join of two paths after it, where the compiler could
      // copy the registers before the wait)
      if ((wpend || (GN_PART_N == 1 && slice > 0)) && pos - pos0 < (uint32_t)RD)
        __builtin_amdgcn_s_waitcnt(0x0F70); // vmcnt(0)
      if constexpr (GN_WCACHE) GN_WC_WAIT(RWAIT_PV);
      if constexpr (GN_PART_N == 1) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(pv) : "n"(RWAIT_PV));
    }
    // (SL > 1: the cached bucket first, as bit 8 of mm; the others load the cache when they come)
    uint32_t mm = SL > 1 && ((bm >> cb) & 1) ? (bm ^ (1u << cb)) | 256u : bm;
#pragma unroll 1
    while (mm) {
      int b;
      if (mm & 256u) b = cb, mm ^= 256u;
      else b = __builtin_ctz(mm), mm &= mm - 1;
      const int buf = (int)(bq & 1);
      int tl = tid;
      asm volatile("" : "+v"(tl));
      const int ln = tl & 63, row = ln & 15, kg = ln >> 4;
      if constexpr (SL > 1 && GN_WCACHE) {
        if (b != cb) { // a tile's second bucket: the cache's fill now, behind the ring's loads
          cb = b;
          wc_load(b);
          GN_WC_WAIT(0);
        }
        const uint8_t *xa = xt + row * XS + kg * 16 + 64 * KPW * wave;
        int4v acc = {0, 0, 0, 0};
        constexpr int FB = 2;
        int stop = 0;
        asm volatile("" : "+s"(stop));
#pragma unroll
        for (int k0 = 0; k0 < KPW && !stop; k0 += FB) {
          int4v av[FB];
#pragma unroll
          for (int j = 0; j < FB; ++j) av[j] = *reinterpret_cast<const int4v *>(xa + 64 * (k0 + j));
#pragma unroll
          for (int j = 0; j < FB; ++j) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[j], wc[k0 + j], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(&acc0[buf][(4 * kg + i) * AS + row], acc[i]);
      } else {
        const uint8_t *xa = xt + row * XS + kg * 16 + 64 * KPW * wave;
        // (w0f: the k-step's 64 lanes x 16 B are one contiguous 1 KiB)
        // (SL > 1: wave w of perspective h covers the net's k-steps of its slice of that side)
        constexpr int WH = NW / 2;
        const int wsl = SL > 1 ? (wave / WH) * WH * SL + slice * WH + wave % WH : wave;
#ifdef GN_AB_W0_FIXED // timing diagnostics only (wrong results): every k-step's weights from one 1-KiB block
        const int8_t *wb = net.w0f + (size_t)ln * 16;
        constexpr int WSTEP = 0;
#else
        const int8_t *wb = net.w0f + (((size_t)b * KSF + KPW * wsl) * 64 + ln) * 16;
        constexpr int WSTEP = 1024;
#endif
        int4v acc = {0, 0, 0, 0};
        // (batches of FB k-steps: the next tile's rows stay in flight in registers meanwhile)
        // (`stop`, always 0, is opaque to the compiler: without a runtime exit test it schedules the
        // fully unrolled loop's loads so that the kernel spills 20 VGPRs, a 3 % slower stream;
        // tests/test_host.py::test_stream_kernel_does_not_spill)
        constexpr int FB = 2;
        int stop = 0;
        asm volatile("" : "+s"(stop));
#pragma unroll
        for (int k0 = 0; k0 < KPW && !stop; k0 += FB) {
          int4v wv[FB], av[FB];
#pragma unroll
          for (int j = 0; j < FB; ++j) wv[j] = *reinterpret_cast<const int4v *>(wb + WSTEP * (k0 + j));
#pragma unroll
          for (int j = 0; j < FB; ++j) av[j] = *reinterpret_cast<const int4v *>(xa + 64 * (k0 + j));
#pragma unroll
          for (int j = 0; j < FB; ++j) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[j], wv[j], acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(&acc0[buf][(4 * kg + i) * AS + row], acc[i]);
      }
#ifndef GN_AB_NO_BARRIER
      __syncthreads();
#endif
      // a position's output index (parent P, or np + its child index) and whether it is evaluated
      // in bucket b
      auto present = [&](int pos) -> bool {
        const uint32_t m = (mw[pos >> 2] >> (8 * (pos & 3))) & 0xFF;
        return (m & 1) && (int)((m >> 1) & 7) == b;
      };
      auto out_index = [&](int pos, int adjv) -> uint64_t {
        const uint32_t P = p_first + (uint32_t)__builtin_popcount(pm & ((2u << pos) - 1)) - (pm & 1);
        return ((pm >> pos) & 1) ? (uint64_t)P : (uint64_t)np + (u0 + pos - P - 1 + adjv);
      };
      if constexpr (SL > 1) {
        if (wave == (int)(bq % NW)) { // this slice's fc_0 sums of bucket b to its partial array
          // the tile's 16 adj values by one scalar load (the descriptor is in the scalar cache
          // since the tile's start): a vector load here would make the compiler wait for every
          // vector load in flight, i.e. the ring's next entries (in-order vmcnt)
          // lane = (position wp, outputs 4 wj .. 4 wj + 3): one 16-B load of the sums and one
          // 16-B store per lane (a store is a vector-memory operation younger than the ring's
          // entries in flight, which the next entries' waits then also wait for: one, not four)
          const int wp = ln >> 2, wj = ln & 3;
          const int adjv = adj_of(D, wp);
          int4v *src = reinterpret_cast<int4v *>(&acc0[buf][wp * AS + 4 * wj]);
          if (present(wp)) {
            const uint64_t q = out_index(wp, adjv);
            int4v v = *src;
            if (GN_PART_N == 1 && slice > 0) {
#pragma unroll
              for (int k = 0; k < 4; ++k) v[k] = wadd(v[k], pv[k]); // (wrapping, as the LDS atomics)
            }
            *reinterpret_cast<int4v *>(part + ((uint64_t)(GN_PART_N == 1 ? 0 : slice) * npos + q) * 16 + 4 * wj) = v;
          }
          *src = int4v{0, 0, 0, 0}; // free for bucket bq + 2
        }
      } else if (wave == (int)(bq % NW)) { // fc_0 activations, fc_1, fc_2, outputs of bucket b
        // the finishing step's scalar weights and the tile's PSQT first (one wait for memory)
        const int32_t bias0 = net.b0[b * 16 + row];
        const int32_t b1l = net.b1[b * 32 + row], b1h = net.b1[b * 32 + 16 + row];
        const int32_t w2l = net.w2[b * 32 + row], w2h = net.w2[b * 32 + 16 + row];
        const int32_t b2v = net.b2[b];
        int2 pq[4] = {};
        int adj[4] = {};
        if (row == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) pq[i] = *reinterpret_cast<const int2 *>(D->psq[4 * kg + i]), adj[i] = D->adj[4 * kg + i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int pos = 4 * kg + i;
          const int32_t vv = wadd(acc0[buf][pos * AS + row], bias0);
          if (row < 15) {
            const long long s2 = ((long long)vv * vv) >> 19;
            in1[buf][pos][row] = (uint8_t)(s2 < 127 ? s2 : 127);
            in1[buf][pos][15 + row] = (uint8_t)clampi(vv >> 6, 0, 127);
          } else {
            fwd[buf][pos] = wmul(vv, 600 * 16) / (127 * 64);
            in1[buf][pos][30] = 0;
            in1[buf][pos][31] = 0;
          }
        }
        ps::wave_sync();
#pragma unroll
        for (int i = 0; i < 4; ++i) acc0[buf][(4 * kg + i) * AS + row] = 0; // free for bucket bq + 2
        const int4v zero = {0, 0, 0, 0};
        // (fc_1's weights by every lane, no branch around the loads: lanes kg >= 2 hold a copy whose
        // products meet the zero A operand)
        const int4v wl = *reinterpret_cast<const int4v *>(net.w1 + ((size_t)b * 32 + row) * 32 + (kg & 1) * 16);
        const int4v wh = *reinterpret_cast<const int4v *>(net.w1 + ((size_t)b * 32 + 16 + row) * 32 + (kg & 1) * 16);
        int4v a1 = zero;
        if (kg < 2) a1 = *reinterpret_cast<const int4v *>(&in1[buf][row][kg * 16]);
        const int4v cl = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, wl, zero, 0, 0, 0);
        const int4v ch = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, wh, zero, 0, 0, 0);
        int32_t l2[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int32_t l = clampi(wadd(cl[i], b1l) >> 6, 0, 127), hh = clampi(wadd(ch[i], b1h) >> 6, 0, 127);
          l2[i] = w2l * l + w2h * hh;
        }
#pragma unroll
        for (int off = 8; off; off >>= 1)
#pragma unroll
          for (int i = 0; i < 4; ++i) l2[i] = wadd(l2[i], __shfl_xor(l2[i], off, 16));
        if (row == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int pos = 4 * kg + i;
            const uint32_t m = (mw[pos >> 2] >> (8 * (pos & 3))) & 0xFF;
            if ((m & 1) && (int)((m >> 1) & 7) == b) {
              const int32_t positional = wadd(wadd(b2v, l2[i]), fwd[buf][pos]);
              const int32_t psqt = (int32_t)((uint32_t)pq[i].x - (uint32_t)pq[i].y) / 2;
              const int2 val = make_int2(psqt / 16, positional / 16);
              const uint32_t P = p_first + (uint32_t)__builtin_popcount(pm & ((2u << pos) - 1)) - (pm & 1);
              if ((pm >> pos) & 1) out_parent[P] = val;
              else out_child[u0 + pos - P - 1 + adj[i]] = val;
            }
          }
        }
      }
      ++bq;
    }
    sp_l += SP_T() - t2;
  }
#ifdef GN_STREAM_PROF
  if ((tid & 63) == 0) {
    SP_ADD(0, sp_s), SP_ADD(1, sp_w), SP_ADD(2, sp_l);
    if (wave == 0) SP_ADD(3, ntiles), SP_ADD(4, sp_m), SP_ADD(5, sp_n);
  }
#else
  (void)sp_s, (void)sp_w, (void)sp_l, (void)sp_m, (void)sp_n, (void)sp_e0, (void)sp_e1;
#endif
  };
  if (hu) run_group(std::integral_constant<int, 1>{});
  else run_group(std::integral_constant<int, 0>{});
  if (use_scr) { // every wave's stores are complete before the slot goes back to the pool
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_fetch_and(pool + 8 * (my_slot / POOL_PER_XCD) + (my_slot % POOL_PER_XCD) / 32,
                             ~(1u << (my_slot % 32)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#ifdef GN_XCD_PROF
  if (tid == 0) {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    x &= 7;
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    atomicMax(&gn_xp[x], t1);
    atomicMin(&gn_xp[8 + x], xp_t0);
    atomicAdd(&gn_xp[16 + x], ntiles ? (unsigned long long)T[ntiles - 1].e_end[0] + T[ntiles - 1].e_end[1] : 0ull);
    atomicAdd(&gn_xp[24 + x], 1ull);
  }
#endif
}

// The column-sliced stream's finish when finalize does not take it over (a thread per position,
// slice_finish_one).  pinfo.y < 0: a position the big net does not evaluate (left as it is).
template <int SL>
__global__ void __launch_bounds__(256) slice_finish_kernel(NetDevice net, const int32_t *__restrict__ part,
                                                           const int2 *__restrict__ pinfo, uint64_t npos, uint32_t np,
                                                           int2 *__restrict__ out_parent, int2 *__restrict__ out_child) {
  __shared__ int4v w1s[8 * 32 * 2];
  stage_fc1(w1s, net);
  __syncthreads();
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= npos) return;
  const int2 info = pinfo[q];
  if (info.y < 0) return;
  const int2 val = slice_finish_one<GN_PART_N>(net, w1s, part, npos, q, info);
  if (q < np) out_parent[q] = val;
  else out_child[q - np] = val;
}

hipError_t launch_plan_stream(const NetDevice &net, const gn_board *parents, size_t n, const uint64_t *offsets,
                              const ChildDelta *deltas, const uint8_t *need_parent, const uint8_t *need_child,
                              int2 *out_parent, int2 *out_child, int swz, const uint8_t *next_slot, int chain_k,
                              int kc, const uint64_t *eoff, uint64_t *ent, TileDesc *tiles, uint32_t *btiles,
                              uint32_t *pool, uint32_t *err, unsigned long long *rows_out,
                              unsigned long long *pads_out, size_t b0, size_t b1, const uint32_t *order,
                              hipEvent_t mid, hipStream_t s, int slices, int32_t *part, size_t npos,
                              int2 *pinfo, hipEvent_t fin, bool finish, int phases) {
  if (!n || b1 <= b0) return hipSuccess;
  const bool do_plan = phases & PLAN_PHASE, do_stream = phases & STREAM_PHASE;
  if (n >= 0x80000000ull) return hipErrorInvalidValue; // 32-bit parent indices in the kernels
  const uint32_t K = chain_k > 1 && next_slot ? (uint32_t)chain_k : 1u;
  const int scr = K > 1 && kc; // the king cache's rows (the chained walk itself needs no scratch)
  if (b1 > (n + K - 1) / K) return hipErrorInvalidValue;
  const uint32_t nb = (uint32_t)(b1 - b0), B0 = (uint32_t)b0, B1 = (uint32_t)b1;
  const unsigned pg = (nb + PLAN_WAVES - 1) / PLAN_WAVES, g = swz == 1 ? 8 * ((nb + 7) / 8) : nb + nb / 16 + 8; // (stream_eval_kernel: claims)
  if (net.L1 == 3072) {
    const bool sliced = slices == 3 && part && pinfo;
    if (do_plan) {
      if (sliced) { // (positions the big net does not evaluate keep pinfo.y < 0; the plan writes the rest)
        hipError_t e = hipMemsetAsync(pinfo, 0xFF, npos * sizeof(int2), s);
        if (e != hipSuccess) return e;
      }
      hipLaunchKernelGGL((plan_kernel<3072>), dim3(pg), dim3(GN_FRONT_WG), 0, s, net, parents, offsets, deltas, need_parent,
                         need_child, K > 1 ? next_slot : nullptr, (uint32_t)n, K, B0, B1, K > 1 ? kc : 0, eoff, ent,
                         tiles, btiles, rows_out, pads_out, err, sliced ? pinfo : nullptr,
                         sliced ? ps::field_xu(3072, 3) : ps::field_xu(3072, 1), sliced ? ps::field_hu(3072, 3) : ps::field_hu(3072, 1));
      if (mid) (void)hipEventRecord(mid, s);
    }
    if (!do_stream) {
    } else if (sliced) { // three launches over 1,024 columns each (claim counters pool[64 + 8 slice ..]),
      // then the finish
      for (int sl = 0; sl < 3; ++sl)
        hipLaunchKernelGGL((stream_eval_kernel<3072, 3>), dim3(g), dim3(128), 0, s, net, offsets, (uint32_t)n, K, B0,
                           B1, swz, eoff, ent, tiles, btiles, order, out_parent, out_child, pool, scr, err,
                           pool + 64 + 8 * sl, sl, part, (uint64_t)npos, pinfo);
      if (fin) (void)hipEventRecord(fin, s);
      if (finish) // (otherwise the caller's finalize takes the outputs from part itself)
        hipLaunchKernelGGL((slice_finish_kernel<3>), dim3((unsigned)((npos + 255) / 256)), dim3(256), 0, s, net, part,
                           pinfo, (uint64_t)npos, (uint32_t)n, out_parent, out_child);
    } else {
      hipLaunchKernelGGL((stream_eval_kernel<3072>), dim3(g), dim3(384), 0, s, net, offsets, (uint32_t)n, K, B0, B1,
                         swz, eoff, ent, tiles, btiles, order, out_parent, out_child, pool, scr, err, pool + 64, 0,
                         nullptr, (uint64_t)0, nullptr);
      if (fin) (void)hipEventRecord(fin, s);
    }
  } else if (net.L1 == 1024) {
    if (do_plan) {
      hipLaunchKernelGGL((plan_kernel<1024>), dim3(pg), dim3(GN_FRONT_WG), 0, s, net, parents, offsets, deltas, need_parent,
                         need_child, K > 1 ? next_slot : nullptr, (uint32_t)n, K, B0, B1, K > 1 ? kc : 0, eoff, ent,
                         tiles, btiles, rows_out, pads_out, err, nullptr, ps::field_xu(1024, 1), ps::field_hu(1024, 1));
      if (mid) (void)hipEventRecord(mid, s);
    }
    if (do_stream) {
      hipLaunchKernelGGL((stream_eval_kernel<1024>), dim3(g), dim3(128), 0, s, net, offsets, (uint32_t)n, K, B0, B1,
                         swz, eoff, ent, tiles, btiles, order, out_parent, out_child, pool, scr, err, pool + 64, 0,
                         nullptr, (uint64_t)0, nullptr);
      if (fin) (void)hipEventRecord(fin, s);
    }
  } else {
    return hipErrorInvalidValue;
  }
#ifdef GN_PLAN_PROF
  {
    unsigned long long c[4];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(gn_pp), sizeof(c));
    fprintf(stderr, "plan prof: wave-cycles setup %llu slots %llu delta puts %llu king jobs %llu\n", c[0], c[1],
            c[2], c[3]);
    memset(c, 0, sizeof(c));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gn_pp), c, sizeof(c));
  }
#endif
#ifdef GN_XCD_PROF
  {
    unsigned long long c[32];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(gn_xp), sizeof(c));
    unsigned long long t0 = ~0ull;
    for (int x = 0; x < 8; ++x) t0 = c[8 + x] < t0 ? c[8 + x] : t0;
    fprintf(stderr, "xcd prof:");
    for (int x = 0; x < 8; ++x)
      fprintf(stderr, " [%d] end %.2f ms start %.2f ms entries %llu wgs %llu;", x, (c[x] - t0) * 1e-5,
              (c[8 + x] - t0) * 1e-5, c[16 + x], c[24 + x]);
    fprintf(stderr, "\n");
    for (int x = 0; x < 8; ++x) c[x] = 0, c[8 + x] = ~0ull, c[16 + x] = 0, c[24 + x] = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gn_xp), c, sizeof(c));
  }
#endif
#ifdef GN_STREAM_PROF
  {
    unsigned long long c[8];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(c, HIP_SYMBOL(gn_sp), sizeof(c));
    fprintf(stderr, "stream prof: wave-cycles stream %llu barrier %llu ls %llu; tiles %llu; "
                    "entries max-list %llu sum %llu (balance %.3f), no-op entries %llu scratch-order + %llu tile-end\n",
            c[0], c[1], c[2], c[3], c[4], c[5], c[5] ? 2.0 * c[4] / c[5] : 0.0, c[6], c[7]);
    memset(c, 0, sizeof(c));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(gn_sp), c, sizeof(c));
  }
#endif
  return hipGetLastError();
}

} // namespace gn
