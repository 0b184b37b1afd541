// kernels.hip — gfx950 kernels of libgpu_nnue.
//
// eval_net<L1, PAR>   the hot path: HalfKAv2_hm feature-transformer gather-
//                     accumulate (int16 rows, wrapping adds) + transform +
//                     the bucket-grouped int8 MFMA layer stack, one 16-position
//                     tile per workgroup.
// classify / reeval / finalize   Eval::evaluate.
// count / write children, count_sum   legal movegen for expansion and perft.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "device_util.h"
#include "kernels.h"

#ifndef GN_SMALL_DEPTH
#define GN_SMALL_DEPTH 4 // eval_net<128>: FT rows in flight per thread (8 at 5 waves per SIMD: 0.72 ms, 6 at 6: 0.64, 4 at 8: 0.555)
#endif
#ifndef GN_SMALL_WPE
#define GN_SMALL_WPE 8 // eval_net<128>: waves per SIMD (64 VGPRs)
#endif


namespace gn {

// ------------------------------------------------------------ layer stack --
// NetworkArchitecture::propagate for a 16-position tile held in LDS as
// transformed features xt[16][L1 + 16] (u8).  Per distinct bucket b in the
// tile (sequentially, all waves together):
//   fc_0  [16 x L1] . [L1 x 16]: the L1/64 k-steps of int8 MFMA 16x16x64 are
//         split across the NW waves (all weight loads of a wave in flight at
//         once); partial 16x16 int32 tiles are summed with LDS integer atomics
//         (exact and order-independent);
//   wave 0: SqrClippedReLU / ClippedReLU -> in1[16][32], fc_1 [16 x 32] .
//         [32 x 32] as two MFMAs (K zero-padded to 64), fc_2 by a 16-lane
//         shuffle reduction, + the skip term from fc_0[15].
// Lane layout of v_mfma_i32_16x16x64_i8: lane l holds A[row l&15][16(l>>4)..+16],
// B[16(l>>4)..+16][col l&15]; C[4(l>>4)+i][l&15] in acc[i].  The K grouping
// inside a lane is irrelevant to the result as long as A and B use the same.
// ls: LDS scratch of LS_SCRATCH bytes.  valid(pos, b): slot pos holds a
// position of bucket b; emit(pos, {psqt/16, positional/16}).
constexpr int LS_SCRATCH = 16 * 16 * 4 + 16 * 32 + 16 * 4; // acc + in1 + fwd = 1600 B

template <int L1, int NW, class Valid, class Emit>
__device__ __forceinline__ void layer_stack_tile(const NetDevice &net, const uint8_t *xt, uint8_t *ls,
                                                 const int32_t (*psq)[2], int tid, uint32_t bm,
                                                 Valid &&valid, Emit &&emit) {
  constexpr int XS = L1 + 16, KS = L1 / 64;
  int32_t *acc0 = reinterpret_cast<int32_t *>(ls);                 // [16 pos][16 out]
  uint8_t(*in1)[32] = reinterpret_cast<uint8_t(*)[32]>(ls + 1024); // [16][32]
  int32_t *fwd = reinterpret_cast<int32_t *>(ls + 1536);           // [16]
  const int lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kg = lane >> 4;
  uint32_t m = bm;
  while (m) {
    const int b = __builtin_ctz(m);
    m &= m - 1;
    for (int i = tid; i < 256; i += NW * 64) acc0[i] = 0;
    __syncthreads();
    {
      int4v acc = {0, 0, 0, 0};
      const uint8_t *xa = xt + row * XS + kg * 16;
      // big nets: w0f (nnue.h: 1 KiB per k-step, 176 -> 166 ms on configs[2]); the small net's two
      // k-steps keep the row-major w0 (its 16 rows are one 2 KiB block; w0f measured 6 % slower)
      constexpr bool FRAG = L1 > 128;
      const int8_t *wb = FRAG ? net.w0f + ((size_t)b * KS * 64 + lane) * 16 : net.w0 + ((size_t)b * 16 + row) * L1 + kg * 16;
      bool any = false;
#pragma unroll
      for (int t = 0; t < (KS + NW - 1) / NW; ++t) {
        const int ks = wave + t * NW;
        if (KS % NW == 0 || ks < KS) { // static when the k-steps split evenly: all loads issue together
          const int4v a = *reinterpret_cast<const int4v *>(xa + 64 * ks);
          const int4v w = *reinterpret_cast<const int4v *>(wb + (FRAG ? 1024 : 64) * ks);
          acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, w, acc, 0, 0, 0);
          any = true;
        }
      }
      if (any) {
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(&acc0[(4 * kg + i) * 16 + row], acc[i]);
      }
    }
    __syncthreads();
    if (wave == 0) {
      const int32_t bias0 = net.b0[b * 16 + row];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pos = 4 * kg + i;
        const int32_t v = wadd(acc0[pos * 16 + row], bias0);
        if (row < 15) {
          const long long s2 = ((long long)v * v) >> 19;
          in1[pos][row] = (uint8_t)(s2 < 127 ? s2 : 127);
          in1[pos][15 + row] = (uint8_t)clampi(v >> 6, 0, 127);
        } else {
          fwd[pos] = wmul(v, 600 * 16) / (127 * 64);
          in1[pos][30] = 0;
          in1[pos][31] = 0;
        }
      }
    }
    __syncthreads();
    if (wave == 0) {
      const int4v zero = {0, 0, 0, 0};
      int4v a = zero, wl = zero, wh = zero;
      if (kg < 2) {
        a = *reinterpret_cast<const int4v *>(&in1[row][kg * 16]);
        wl = *reinterpret_cast<const int4v *>(net.w1 + ((size_t)b * 32 + row) * 32 + kg * 16);
        wh = *reinterpret_cast<const int4v *>(net.w1 + ((size_t)b * 32 + 16 + row) * 32 + kg * 16);
      }
      const int4v cl = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, wl, zero, 0, 0, 0);
      const int4v ch = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, wh, zero, 0, 0, 0);
      const int32_t b1l = net.b1[b * 32 + row], b1h = net.b1[b * 32 + 16 + row];
      const int32_t w2l = net.w2[b * 32 + row], w2h = net.w2[b * 32 + 16 + row];
      int32_t part[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int32_t l = clampi(wadd(cl[i], b1l) >> 6, 0, 127), hh = clampi(wadd(ch[i], b1h) >> 6, 0, 127);
        part[i] = w2l * l + w2h * hh;
      }
#pragma unroll
      for (int off = 8; off; off >>= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) part[i] = wadd(part[i], __shfl_xor(part[i], off, 16));
      if (row == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int pos = 4 * kg + i;
          if (valid(pos, b)) {
            const int32_t positional = wadd(wadd(net.b2[b], part[i]), fwd[pos]);
            const int32_t psqt = (int32_t)((uint32_t)psq[pos][0] - (uint32_t)psq[pos][1]) / 2;
            emit(pos, make_int2(psqt / 16, positional / 16));
          }
        }
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------- material (Eval) --
struct Material {
  int pawns[2], npm[2];
};

__device__ __forceinline__ Material material(const Board &B, const gn_eval_params &P) {
  Material m;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const Bitboard o = B.byColor[c];
    m.pawns[c] = popcnt(B.byType[PAWN] & o);
    m.npm[c] = P.piece_value[1] * popcnt(B.byType[KNIGHT] & o) + P.piece_value[2] * popcnt(B.byType[BISHOP] & o) +
               P.piece_value[3] * popcnt(B.byType[ROOK] & o) + P.piece_value[4] * popcnt(B.byType[QUEEN] & o);
  }
  return m;
}

// --------------------------------------------------------------- eval_net --
// Workgroup = 2 * G * PAR threads, G = L1 / 16 threads per (position,
// perspective): thread j of a perspective group owns accumulator columns
// [8j, 8j+8) and [L1/2 + 8j, L1/2 + 8j + 8), so the transform's pairwise
// product needs no data exchange.  Big net: G = 192, PAR = 1 (384 threads, the
// 16 positions of the tile one after another); small net: G = 8, PAR = 16
// (256 threads, all 16 positions at once).
template <int L1, int PAR, bool CLS = false>
__global__ void __launch_bounds__(2 * (L1 / 16) * PAR) __attribute__((amdgpu_waves_per_eu(PAR == 1 ? 1 : GN_SMALL_WPE)))
    eval_net_kernel(NetDevice net, const gn_board *__restrict__ boards, const uint8_t *__restrict__ need,
                    size_t n, int2 *__restrict__ out, const uint32_t *__restrict__ perm, unsigned tiles, int swz,
                    unsigned long long *__restrict__ rows_out, unsigned tn, gn_eval_params P,
                    uint8_t *__restrict__ need_small, uint8_t *__restrict__ need_big) {
  static_assert(!CLS || PAR > 1, "the folded selection is the small net's (mode FULL)");
  constexpr int G = L1 / 16;
  constexpr int NT = 2 * G * PAR;
  constexpr int NW = NT / 64;
  constexpr int TILE = 16;
  constexpr int XS = L1 + 16; // padded LDS row: conflict-free ds_read_b128 across 16 rows
  constexpr uint32_t RS = ft_row_stride(L1);
  static_assert(NT % 64 == 0 && TILE % PAR == 0, "geometry");

  // LDS: big net 53.2 KB -> 3 workgroups (18 waves) per CU.  The feature list
  // (phase 0-1) and the layer-stack scratch (phase 2) share one region.
  constexpr int ROWS_BYTES = TILE * 2 * 32 * 2;
  constexpr int SCRATCH = ROWS_BYTES > LS_SCRATCH ? ROWS_BYTES : LS_SCRATCH;
  __shared__ __attribute__((aligned(16))) uint8_t xt[TILE * XS];
  __shared__ __attribute__((aligned(16))) uint8_t scratch[SCRATCH];
  __shared__ int32_t psq[TILE][2];
  __shared__ int nfeat[TILE];
  __shared__ int bkt[TILE];
  __shared__ uint32_t bmask;
  __shared__ uint32_t gidx[TILE];
  __shared__ uint8_t sstm[TILE];
  __shared__ uint8_t refpc[64];     // piece per square of the tile's first position (0xFF: none)
  __shared__ uint32_t cmask[2];     // squares holding the same piece in every valid position
  __shared__ uint16_t crow[2][32];  // the tile's common rows by ABSOLUTE perspective
  __shared__ int ccnt;
  __shared__ gn_board tb[TILE];     // the tile's boards (a dead slot: zeroed, occ 0)
  __shared__ uint32_t tix[TILE];    // their batch indices
  uint16_t(*rows)[2][32] = reinterpret_cast<uint16_t(*)[2][32]>(scratch);

  const int tid = threadIdx.x;
  // XCD-aware tile order: blocks b, b+8, ... share an XCD (round-robin
  // dispatch); give each XCD a contiguous range of tiles so its 4 MiB L2 sees
  // positions of similar king squares (after an optional king sort).
  unsigned tile = blockIdx.x;
  if (swz) {
    const unsigned t8 = (tiles + 7) / 8;
    tile = (blockIdx.x & 7) * t8 + (blockIdx.x >> 3);
    if (tile >= tiles) return;
  }
  // tn positions per workgroup (16; fewer for a small batch: the big net's phase 1 walks a tile's
  // positions one after another, so a 128-position batch in 16-position tiles is 8 workgroups each
  // 16 gathers deep -- the drop-in's latency -- while 2-position tiles are 64 workgroups 2 deep)
  const size_t base = (size_t)tile * tn;
  // the tile's boards to LDS by tn lanes in one round trip (perm, need, board), instead of a
  // dependent board load per position in each phase-0 loop below (slots >= tn: empty boards)
  if (tid < TILE) {
    const size_t q = base + tid;
    const bool in = (unsigned)tid < tn && q < n;
    const size_t i = in ? (perm ? perm[q] : q) : 0;
    gn_board b = {};
    if (CLS) {
      // mode FULL's selection folded in (classify_kernel): the small net evaluates the positions
      // whose |simple_eval| exceeds the threshold, the rest go to the big net; the small net's
      // re-evaluation rule is applied where its outputs are written (emit, below)
      if (in) {
        Board B;
        uint8_t sm = 0, bg = 0;
        const gn_board g = boards[i];
        if (unpack(g, B)) {
          const Material m = material(B, P);
          const int us = B.stm;
          const int simple = P.piece_value[0] * (m.pawns[us] - m.pawns[us ^ 1]) + (m.npm[us] - m.npm[us ^ 1]);
          sm = abs(simple) > P.small_net_threshold;
          bg = !sm;
        }
        need_small[i] = sm;
        need_big[i] = bg;
        if (sm) b = g;
      }
    } else if (in && (!need || need[i])) {
      b = boards[i];
    }
    tb[tid] = b;
    tix[tid] = (uint32_t)i;
  }
  __syncthreads();
  auto pos_index = [&](int sl) -> size_t { return tix[sl]; };
  auto pos_live = [&](int sl, size_t) { return tb[sl].occ != 0; }; // (a live board without pieces has no features either)

  // ---- phase 0: feature rows of both ABSOLUTE perspectives, one wave per position.
  // Common-row base: the rows of the pieces that stand on the same square in every
  // valid position of the tile (both kings included, so their feature indices agree)
  // are gathered once per tile into the accumulator's starting value instead of once
  // per position.  With the batch sorted by (kings, first squares' pieces) tiles share
  // their kings and a few unmoved pieces.  Wrapping int16 adds are order-independent,
  // so the results are those of a plain refresh.
  // Big net only (PAR == 1): the small net's table is L2-resident and its rows cheap, so
  // the two extra barriers cost more than the rows they save.
  constexpr bool CB = PAR == 1;
  {
    const int lane = tid & 63, wave = tid >> 6;
    if (!CB) {
      if (tid == 0) bmask = 0;
    } else {
      if (wave == 0) { // A: the first position's placement is the reference
        const size_t i = pos_index(0);
        int pc = 0xFF;
        if (pos_live(0, i)) {
          const gn_board p = tb[0];
          if (wave_features(p, nullptr, nullptr, lane)) pc = lane_piece(p, lane);
        }
        refpc[lane] = (uint8_t)pc;
        if (lane == 0) bmask = 0, cmask[0] = ~0u, cmask[1] = ~0u;
      }
      __syncthreads();
      for (int sl = wave; sl < TILE; sl += NW) { // B: AND of the per-position agreement masks
        const size_t i = pos_index(sl);
        if (!pos_live(sl, i)) continue;
        const gn_board p = tb[sl];
        const int pc = lane_piece(p, lane);
        const uint64_t eq = __ballot(pc == refpc[lane]);
        if (wave_features(p, nullptr, nullptr, lane) && lane == 0) {
          atomicAnd(&cmask[0], (uint32_t)eq);
          atomicAnd(&cmask[1], (uint32_t)(eq >> 32));
        }
      }
    }
    __syncthreads();
    // C: the common squares (occupied in the reference, both kings among them, else none)
    const int rp = CB ? refpc[lane] : 0;
    const bool cm = CB && ((((uint64_t)cmask[1] << 32 | cmask[0]) >> lane) & 1) && rp != 0 && rp != 0xFF;
    const uint64_t wkb = __ballot(cm && rp == make_piece(WHITE, KING));
    const uint64_t bkb = __ballot(cm && rp == make_piece(BLACK, KING));
    const uint64_t excl = wkb && bkb ? __ballot(cm) : 0;
    if (wave == 0) {
      if ((excl >> lane) & 1) {
        const int k = popcnt(excl & ((1ull << lane) - 1));
        crow[WHITE][k] = (uint16_t)feature_index(WHITE, lane, rp, __builtin_ctzll(wkb));
        crow[BLACK][k] = (uint16_t)feature_index(BLACK, lane, rp, __builtin_ctzll(bkb));
      }
      if (lane == 0) ccnt = popcnt(excl);
    }
    for (int sl = wave; sl < TILE; sl += NW) {
      const size_t i = pos_index(sl);
      int cnt = 0, stm = 0;
      if (pos_live(sl, i)) {
        const gn_board p = tb[sl];
        stm = p.stm_ep >> 7;
        // big net: rows by absolute perspective (the base is per colour); small net: by
        // relative perspective (h = 0: side to move), as the transform consumes them
        if constexpr (CB) cnt = wave_features_excl(p, rows[sl][WHITE], rows[sl][BLACK], lane, excl);
        else cnt = wave_features(p, rows[sl][stm], rows[sl][stm ^ 1], lane);
      }
      if (lane == 0) {
        gidx[sl] = (uint32_t)i;
        nfeat[sl] = cnt;
        bkt[sl] = cnt ? (cnt - 1) / 4 : 0;
        sstm[sl] = (uint8_t)stm;
        if (cnt) atomicOr(&bmask, 1u << ((cnt - 1) / 4));
      }
    }
  }
  __syncthreads();
  if (rows_out && tid == 0) { // FT rows this tile gathers: common rows once, then each position's own
    unsigned long long r = 0;
    int any = 0;
    for (int sl = 0; sl < TILE; ++sl)
      if (nfeat[sl]) r += (unsigned long long)(nfeat[sl] - ccnt), any = 1;
    if (any) atomicAdd(rows_out, 2ull * (r + (unsigned long long)ccnt));
  }

  // ---- phase 1: gather-accumulate + transform into the LDS tile (h: absolute perspective
  // for the big net, relative for the small net)
  {
    const int q = tid / (2 * G), h = (tid / G) & 1, j = tid % G;
    const uint32_t j16 = 16 * j; // byte offset of this thread's columns in a row
    const int nc = ccnt;
    const uint16_t *cr = crow[h];
    // rows rr[0..cnt) added to lo/hi and, on lane j == 0 when wps, their PSQT at the position's
    // bucket to ps, read from the bucket-major copy pt = net.psqt + bucket * FT_ROWS (90 KB per
    // bucket, its lines shared by all the rows of a king bucket) rather than the row's own PSQT
    // part, a line of its own per row (a third line per row for the small net, whose weights are
    // two); D rows in flight (big net 4: more cost a wave per SIMD; small net GN_SMALL_DEPTH), the
    // tail as one batch (no serialized round trips)
    constexpr int D = PAR == 1 ? 4 : GN_SMALL_DEPTH;
    auto gather = [&](const uint16_t *rr, int cnt, ushort8 &lo, ushort8 &hi, uint32_t &ps, const int32_t *pt,
                      bool wps) {
      int k = 0;
      for (; k + D <= cnt; k += D) {
        ushort8 a[D], b[D];
        uint32_t o[D];
#pragma unroll
        for (int i = 0; i < D; ++i) o[i] = ft_row(rr[k + i]) * RS;
#pragma unroll
        for (int i = 0; i < D; ++i) a[i] = ldft(net.ft, j16 + o[i]);
#pragma unroll
        for (int i = 0; i < D; ++i) b[i] = ldft(net.ft, j16 + o[i] + L1);
        if (wps && j == 0) {
#pragma unroll
          for (int i = 0; i < D; ++i) ps += (uint32_t)pt[ft_row(rr[k + i])];
        }
#pragma unroll
        for (int i = 0; i + 1 < D; i += 2) lo += a[i] + a[i + 1], hi += b[i] + b[i + 1];
        if constexpr (D % 2) lo += a[D - 1], hi += b[D - 1]; // (an odd depth's last row)
      }
      if (k < cnt) { // tail of 1 .. D - 1 rows (indices past the end repeat row k, not added)
        ushort8 a[D - 1], b[D - 1];
        uint32_t o[D - 1], q[D - 1];
#pragma unroll
        for (int i = 0; i < D - 1; ++i) o[i] = ft_row(rr[k + i < cnt ? k + i : k]) * RS;
#pragma unroll
        for (int i = 0; i < D - 1; ++i) a[i] = ldft(net.ft, j16 + o[i]), b[i] = ldft(net.ft, j16 + o[i] + L1);
#pragma unroll
        for (int i = 0; i < D - 1; ++i) q[i] = wps && j == 0 ? (uint32_t)pt[ft_row(rr[k + i < cnt ? k + i : k])] : 0u;
#pragma unroll
        for (int i = 0; i < D - 1; ++i)
          if (k + i < cnt) lo += a[i], hi += b[i], ps += q[i];
      }
    };
    // the tile's starting accumulator: bias + common rows (PSQT per position below)
    ushort8 base_lo = *reinterpret_cast<const ushort8 *>(net.bias + 8 * j);
    ushort8 base_hi = *reinterpret_cast<const ushort8 *>(net.bias + L1 / 2 + 8 * j);
    {
      uint32_t unused = 0;
      gather(cr, nc, base_lo, base_hi, unused, nullptr, false);
    }
#pragma unroll 1
    for (int r = 0; r < TILE / PAR; ++r) {
      const int p = r * PAR + q;
      const int cnt = nfeat[p];
      if (!cnt) continue;
      ushort8 lo = base_lo, hi = base_hi;
      uint32_t ps = 0;
      const int32_t *pt = net.psqt + (size_t)bkt[p] * FT_ROWS;
      if (j == 0) { // PSQT of the common rows at this position's bucket (one lane)
        for (int k = 0; k < nc; ++k) ps += (uint32_t)pt[ft_row(cr[k])];
      }
      gather(rows[p][h], cnt - nc, lo, hi, ps, pt, true);
      // transform: clamp to [0, 254] in the doubled domain, product / 512
      const int rel = CB ? h ^ sstm[p] : h; // 0: side to move
      *reinterpret_cast<uint2 *>(xt + p * XS + rel * (L1 / 2) + 8 * j) = transform8(lo, hi);
      if (j == 0) psq[p][rel] = (int32_t)ps;
    }
  }
  __syncthreads();

  // ---- phase 2: layer stack (MFMA).  Big net: every wave takes part in each bucket's fc_0
  // (48 k-steps); small net (2 k-steps): one wave per bucket present runs the whole stack
  // (layer_stack_wave: no LDS partial sums, no further barrier), the other waves are done
  auto valid = [&](int pos, int b) { return (unsigned)pos < tn && base + pos < n && nfeat[pos] && bkt[pos] == b; };
  auto emit = [&](int pos, int2 v) {
    out[gidx[pos]] = v;
    if (CLS) { // (reeval_kernel's rule)
      const int32_t nnue = wadd(wmul(P.psqt_weight, v.x), wmul(P.positional_weight, v.y)) / 128;
      if (abs(nnue) < P.reeval_threshold) need_big[gidx[pos]] = 1;
    }
  };
  if constexpr (PAR == 1) {
    layer_stack_tile<L1, NW>(net, xt, scratch, psq, (int)threadIdx.x, bmask, valid, emit);
  } else {
    __shared__ __attribute__((aligned(16))) uint8_t lin1[NW][16][32];
    __shared__ int32_t lfwd[NW][16];
    const int lane = tid & 63, wave = tid >> 6;
    int idx = 0;
    for (uint32_t m = bmask; m; m &= m - 1, ++idx)
      if (idx % NW == wave) layer_stack_wave<L1>(net, xt, lin1[wave], lfwd[wave], psq, __builtin_ctz(m), lane, valid, emit);
  }
}

// ---------------------------------------------------------- expand_eval --
// One row program of a slot perspective: lo/hi (and, on psq lanes, ps) -=
// rows rr[k] for k < ns, += rows rr[k] for ns <= k < n; up to 4 rows in flight,
// no loads for absent entries.  save: the batch holding entry 0 also stores
// base = (accumulator before it) - row(rr[0]) (the sibling cache of expand_eval).
template <int L1, bool U>
__device__ __forceinline__ void run_rows(const uint8_t *__restrict__ ft, uint32_t j16, const uint16_t *rr, int k,
                                         int ns, int n, bool psl, uint32_t psb, bool save, ushort8 &base_lo,
                                         ushort8 &base_hi, ushort8 &lo, ushort8 &hi, uint32_t &ps) {
  constexpr uint32_t RS = ft_row_stride(L1);
#pragma unroll 1
  for (; k < n; k += 4) {
    ushort8 a0, a1, a2, a3, b0, b1, b2, b3;
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;
    const uint32_t o0 = (uint32_t)uni<U>(ft_row(rr[k])) * RS;
    a0 = ldft(ft, j16 + o0), b0 = ldft(ft, j16 + o0 + L1);
    if (psl) p0 = ldpd(ft, o0 + psb);
    if (k + 1 < n) {
      const uint32_t o1 = (uint32_t)uni<U>(ft_row(rr[k + 1])) * RS;
      a1 = ldft(ft, j16 + o1), b1 = ldft(ft, j16 + o1 + L1);
      if (psl) p1 = ldpd(ft, o1 + psb);
    }
    if (k + 2 < n) {
      const uint32_t o2 = (uint32_t)uni<U>(ft_row(rr[k + 2])) * RS;
      a2 = ldft(ft, j16 + o2), b2 = ldft(ft, j16 + o2 + L1);
      if (psl) p2 = ldpd(ft, o2 + psb);
    }
    if (k + 3 < n) {
      const uint32_t o3 = (uint32_t)uni<U>(ft_row(rr[k + 3])) * RS;
      a3 = ldft(ft, j16 + o3), b3 = ldft(ft, j16 + o3 + L1);
      if (psl) p3 = ldpd(ft, o3 + psb);
    }
    if (save && k == 0) base_lo = lo - a0, base_hi = hi - b0;
    if (k < ns) lo -= a0, hi -= b0, ps -= p0;
    else lo += a0, hi += b0, ps += p0;
    if (k + 1 < n) {
      if (k + 1 < ns) lo -= a1, hi -= b1, ps -= p1;
      else lo += a1, hi += b1, ps += p1;
    }
    if (k + 2 < n) {
      if (k + 2 < ns) lo -= a2, hi -= b2, ps -= p2;
      else lo += a2, hi += b2, ps += p2;
    }
    if (k + 3 < n) {
      if (k + 3 < ns) lo -= a3, hi -= b3, ps -= p3;
      else lo += a3, hi += b3, ps += p3;
    }
  }
}

// Incremental evaluation of every legal child of a parent (SURVEY.md §8a row
// a14, "children are derived from the parent accumulator by incremental
// add/sub deltas").  One workgroup per parent (or, persistent, a strided walk
// over parents); slot list = [parent, child_0 .. child_{nc-1}] in tiles of 16.
// Threads are split by ABSOLUTE perspective (h = 0 white, 1 black) because the
// side to move alternates between parent and children; h is mapped to the stm
// / ~stm half of the transformed features per slot.  The parent accumulators
// (refreshed once) stay in registers (big net) or LDS (small net, PAR > 1).
// Each slot perspective runs one row program (run_rows):
//   delta child:  parent - rows(removed) + rows(added)   (1-3 rows each, Dirty);
//                 entry 0 is the mover's from-row, and (parent - that row) is
//                 kept in registers while consecutive siblings move the same piece;
//   king moved:   bias + all rows of that perspective (refresh);
//   parent:       its accumulators as they are.
// Register budget: <= 88 VGPRs so that three 384-thread workgroups (the LDS
// limit) are resident per CU (tools/occupancy_probe.hip: 6-wave workgroups above
// 128 VGPRs run one per CU).
template <int L1, int PAR>
__global__ void __launch_bounds__(2 * (L1 / 16) * PAR) __attribute__((amdgpu_waves_per_eu(4)))
    expand_eval_kernel(NetDevice net, const gn_board *__restrict__ parents, const uint64_t *__restrict__ offsets,
                       const gn_board *__restrict__ children, const ChildDelta *__restrict__ deltas,
                       const uint8_t *__restrict__ need_parent,
                       const uint8_t *__restrict__ need_child, int2 *__restrict__ out_parent,
                       int2 *__restrict__ out_child, size_t n_parents, int swz) {
  constexpr int G = L1 / 16;
  constexpr int NT = 2 * G * PAR;
  constexpr int NW = NT / 64;
  constexpr int TILE = 16;
  constexpr int XS = L1 + 16;
  constexpr uint32_t RS = ft_row_stride(L1);
  constexpr int ROWS_BYTES = TILE * 2 * 32 * 2;
  constexpr int SCRATCH = ROWS_BYTES > LS_SCRATCH ? ROWS_BYTES : LS_SCRATCH;
  constexpr int PACC = PAR > 1 ? 2 * L1 : 8; // shared parent accumulators (small net only)
  constexpr bool U = PAR == 1 && G % 64 == 0; // a perspective group = whole waves
  __shared__ __attribute__((aligned(16))) uint8_t xt[TILE * XS];
  __shared__ __attribute__((aligned(16))) uint8_t scratch[SCRATCH];
  __shared__ __attribute__((aligned(16))) uint16_t pacc_lds[PACC];
  __shared__ __attribute__((aligned(16))) int32_t pps_lds[2][8];
  __shared__ uint16_t prow[2][32];
  __shared__ int32_t psq[TILE][2];
  __shared__ uint8_t nsub[TILE][2], ncnt[TILE][2], usep[TILE][2], sstm[TILE], bkt[TILE], valid[TILE];
  __shared__ int pcount, njobs;
  __shared__ uint8_t jobs[TILE * 2];
  __shared__ uint32_t bmask;
  // the parent board, and the first CDL children's deltas (idx + meta, 20 B each),
  // loaded at parent start together with the parent's own rows so that no tile
  // waits on an HBM round trip for its descriptors
  constexpr int CDL = 64;
  __shared__ gn_board pbd;
  __shared__ uint32_t cdl[CDL][5];
  uint16_t(*rows)[2][32] = reinterpret_cast<uint16_t(*)[2][32]>(scratch);

  const int tid = threadIdx.x;
  const int q = tid / (2 * G), h = (tid / G) & 1, j = tid % G;
  const uint32_t j16 = 16 * j; // byte offset of this thread's columns in a row
  // Persistent when gridDim.x < the virtual grid: workgroup b walks virtual blocks
  // b, b + gridDim.x, ... (gridDim.x is a multiple of 8, so every virtual block of a
  // workgroup maps to the same XCD's parent range, in order)
  const size_t vgrid = swz ? 8 * ((n_parents + 7) / 8) : n_parents;
  for (size_t v = blockIdx.x; v < vgrid; v += gridDim.x) {
    __syncthreads(); // LDS of the previous parent is dead
    // XCD-aware parent order: each XCD takes a contiguous range of parents, so
    // the parents of one game (same kings, mostly the same pieces) and their
    // children share that XCD's L2
    size_t p = v;
    if (swz) {
      const size_t p8 = (n_parents + 7) / 8;
      p = (v & 7) * p8 + (v >> 3);
      if (p >= n_parents) continue;
    }
    const uint64_t off = offsets[p];
    const int total = 1 + (int)(offsets[p + 1] - off);

    // ---- pre-phase: is any slot needed?  parent feature rows (both perspectives),
    // parent board and the first CDL deltas into LDS
    if (tid >= 64 && tid - 64 < (total - 1 < CDL ? total - 1 : CDL)) {
      const uint32_t *src = reinterpret_cast<const uint32_t *>(deltas + off + (tid - 64));
#pragma unroll
      for (int w = 0; w < 5; ++w) cdl[tid - 64][w] = src[w];
    }
    int want = 0;
    for (int qq = tid; qq < total; qq += NT)
      want |= qq == 0 ? (need_parent ? need_parent[p] : 1) : (need_child ? need_child[off + qq - 1] : 1);
    if (tid < 64) {
      const gn_board pb = parents[p];
      const int c = wave_features(pb, prow[0], prow[1], tid);
      if (tid == 0) pcount = c, pbd = pb;
    }
    if (!__syncthreads_or(want)) continue;
    if (!pcount) continue;

    // parent accumulators: bias + all rows (group q == 0), kept for every child; the
    // parent's 8 PSQT sums go to LDS (children read one bucket each)
    ushort8 pacc_lo = *reinterpret_cast<const ushort8 *>(net.bias + 8 * j);
    ushort8 pacc_hi = *reinterpret_cast<const ushort8 *>(net.bias + L1 / 2 + 8 * j);
    if (q == 0) {
      const uint32_t pso = 2 * L1 + 16 * (j & 1); // this thread's 4 PSQT buckets (j < 2 only)
      int4v pps = {0, 0, 0, 0};
      const int cnt = pcount;
#pragma unroll 1
      for (int k = 0; k < cnt; k += 4) {
        const int k1 = k + 1 < cnt ? k + 1 : k, k2 = k + 2 < cnt ? k + 2 : k, k3 = k + 3 < cnt ? k + 3 : k;
        const uint32_t o0 = ft_row(prow[h][k]) * RS, o1 = ft_row(prow[h][k1]) * RS;
        const uint32_t o2 = ft_row(prow[h][k2]) * RS, o3 = ft_row(prow[h][k3]) * RS;
        const ushort8 a0 = ldft(net.ft, j16 + o0), a1 = ldft(net.ft, j16 + o1);
        const ushort8 a2 = ldft(net.ft, j16 + o2), a3 = ldft(net.ft, j16 + o3);
        const ushort8 b0 = ldft(net.ft, j16 + o0 + L1), b1 = ldft(net.ft, j16 + o1 + L1);
        const ushort8 b2 = ldft(net.ft, j16 + o2 + L1), b3 = ldft(net.ft, j16 + o3 + L1);
        if (j < 2) {
          pps += ldps(net.ft, o0 + pso);
          if (k + 1 < cnt) pps += ldps(net.ft, o1 + pso);
          if (k + 2 < cnt) pps += ldps(net.ft, o2 + pso);
          if (k + 3 < cnt) pps += ldps(net.ft, o3 + pso);
        }
        pacc_lo += a0, pacc_hi += b0;
        if (k + 1 < cnt) pacc_lo += a1, pacc_hi += b1;
        if (k + 2 < cnt) pacc_lo += a2, pacc_hi += b2;
        if (k + 3 < cnt) pacc_lo += a3, pacc_hi += b3;
      }
      if (PAR > 1) {
        *reinterpret_cast<ushort8 *>(pacc_lds + h * L1 + 8 * j) = pacc_lo;
        *reinterpret_cast<ushort8 *>(pacc_lds + h * L1 + L1 / 2 + 8 * j) = pacc_hi;
      }
      if (j < 2) *reinterpret_cast<int4v *>(&pps_lds[h][4 * j]) = pps;
    }
    if (PAR > 1) {
      __syncthreads();
      pacc_lo = *reinterpret_cast<const ushort8 *>(pacc_lds + h * L1 + 8 * j);
      pacc_hi = *reinterpret_cast<const ushort8 *>(pacc_lds + h * L1 + L1 / 2 + 8 * j);
    }

    ushort8 base_lo = pacc_lo, base_hi = pacc_hi; // parent minus base_key's row (sibling cache)
    int base_key = -1;

#pragma unroll 1
    for (int t0 = 0; t0 < total; t0 += TILE) {
      // per-lane values are re-derived every tile from an opaque copy of the thread
      // id instead of being hoisted and held live across the kernel (VGPR budget)
      int tl = tid;
      asm volatile("" : "+v"(tl));
      const int qt = tl / (2 * G), ht = (tl / G) & 1, jt = tl % G;
      if (tid == 0) bmask = 0, njobs = 0;
      __syncthreads();
      // ---- phase 0: slot descriptors (one thread per slot) from ChildDelta; king-move
      // refreshes are queued and extracted wave-parallel (lane = square)
      if (tid < TILE) {
        const int qq = t0 + tid;
        int vld = 0, stm = 0, cnt = 2;
        if (qq < total) {
          if (qq == 0) {
            vld = need_parent ? need_parent[p] : 1;
            stm = pbd.stm_ep >> 7, cnt = pcount;
            nsub[tid][0] = nsub[tid][1] = ncnt[tid][0] = ncnt[tid][1] = 0;
            usep[tid][0] = usep[tid][1] = 1;
          } else if ((vld = need_child ? need_child[off + qq - 1] : 1)) {
            ChildDelta cd;
            if (qq - 1 < CDL) {
              uint32_t *dst = reinterpret_cast<uint32_t *>(&cd);
#pragma unroll
              for (int w = 0; w < 5; ++w) dst[w] = cdl[qq - 1][w];
            } else {
              cd = deltas[off + qq - 1];
            }
            stm = (cd.meta >> 10) & 1;
            cnt = (cd.meta >> 14) & 63;
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              if (cd.meta & (1u << (8 + hh))) {
                // king moved: the squares that change, for wave_features_king_move
                rows[tid][hh][0] = cd.idx[hh][0];
                rows[tid][hh][1] = cd.idx[hh][1];
                rows[tid][hh][2] = cd.idx[hh][2];
                rows[tid][hh][3] = cd.idx[hh][3];
                usep[tid][hh] = 0, nsub[tid][hh] = 0, ncnt[tid][hh] = (uint8_t)cnt;
                jobs[atomicAdd(&njobs, 1)] = (uint8_t)(tid | (hh << 4));
              } else {
                const int ns = (cd.meta >> (4 * hh)) & 3, na = (cd.meta >> (4 * hh + 2)) & 3;
                rows[tid][hh][0] = cd.idx[hh][0];
                rows[tid][hh][1] = cd.idx[hh][1];
                rows[tid][hh][ns] = cd.idx[hh][2];
                rows[tid][hh][ns + 1] = cd.idx[hh][3];
                usep[tid][hh] = 1, nsub[tid][hh] = (uint8_t)ns, ncnt[tid][hh] = (uint8_t)(ns + na);
              }
            }
          }
        }
        valid[tid] = (uint8_t)vld;
        sstm[tid] = (uint8_t)stm;
        bkt[tid] = (uint8_t)((cnt - 1) / 4);
        if (vld) atomicOr(&bmask, 1u << ((cnt - 1) / 4));
      }
      __syncthreads();
      {
        const int lane = tid & 63, wave = tid >> 6, nj = njobs;
        for (int jb = wave; jb < nj; jb += NW) {
          const int sl = jobs[jb] & 15, hh = jobs[jb] >> 4;
          uint16_t *rw = rows[sl][hh];
          const int kf = rw[0], kt = rw[1], rf = rw[2], rt = rw[3]; // read by every lane before any writes
          wave_features_king_move(pbd, hh, kf, kt, rf, rt, rw, lane);
        }
      }
      __syncthreads();

      // ---- phase 1: accumulators + transform.  PSQT: thread j == 0 of each
      // perspective sums the slot's own bucket (one dword per row).
#pragma unroll 1
      for (int r = 0; r < TILE / PAR; ++r) {
        const int sl = r * PAR + qt;
        if (!valid[sl]) continue;
        const bool fromp = uni<U>(usep[sl][ht]);
        const int b = uni<U>(bkt[sl]), ns = uni<U>(nsub[sl][ht]), n = uni<U>(ncnt[sl][ht]);
        const uint16_t *rr = rows[sl][ht];
        ushort8 lo, hi;
        uint32_t ps = 0;
        int k = 0;
        bool save = false;
        if (!fromp) {
          lo = *reinterpret_cast<const ushort8 *>(net.bias + 8 * jt);
          hi = *reinterpret_cast<const ushort8 *>(net.bias + L1 / 2 + 8 * jt);
        } else {
          ps = (uint32_t)pps_lds[ht][b];
          if (n > 0 && uni<U>(rr[0]) == base_key) {
            lo = base_lo, hi = base_hi, k = 1;
            if (jt == 0) ps -= ldpd(net.ft, (uint32_t)uni<U>(ft_row(rr[0])) * RS + 2 * L1 + 4 * b);
          } else {
            lo = pacc_lo, hi = pacc_hi, save = n > 0;
          }
        }
        run_rows<L1, U>(net.ft, 16 * jt, rr, k, ns, n, jt == 0, 2 * L1 + 4 * b, save, base_lo, base_hi, lo, hi, ps);
        if (save) base_key = uni<U>(rr[0]);
        const int side = uni<U>(ht == sstm[sl] ? 0 : 1);
        *reinterpret_cast<uint2 *>(xt + sl * XS + side * (L1 / 2) + 8 * jt) = transform8(lo, hi);
        if (jt == 0) psq[sl][side] = (int32_t)ps;
      }
      __syncthreads();

      // ---- phase 2: layer stack
      layer_stack_tile<L1, NW>(net, xt, scratch, psq, tl, bmask, [&](int pos, int bb) {
        return t0 + pos < total && valid[pos] && bkt[pos] == bb;
      }, [&](int pos, int2 val) {
        if (t0 + pos == 0) out_parent[p] = val;
        else out_child[off + t0 + pos - 1] = val;
      });
    }
  }
}

hipError_t launch_eval_net(const NetDevice &net, const gn_board *boards, const uint8_t *need, size_t n, int2 *out,
                           const uint32_t *perm, int swz, hipStream_t s, unsigned long long *rows_out,
                           const gn_eval_params *cls, uint8_t *need_small, uint8_t *need_big) {
  if (cls && (net.L1 != 128 || !need_small || !need_big)) return hipErrorInvalidValue;
  const gn_eval_params P = cls ? *cls : gn_eval_params{};
  if (!n) return hipSuccess;
  // positions per workgroup: 16, or for a big net (positions one after another in phase 1) and a
  // batch of fewer than 32 k positions, as few as keep >= 2,048 workgroups (>= 2; 1 for a batch of
  // <= 1,024 positions, the drop-in's one game per call with its reply levels: p50 0.176 -> 0.169
  // ms, r06s)
  unsigned tn = 16;
#ifndef GN_TN_MIN
#define GN_TN_MIN (n <= 1024 ? 1u : 2u)
#endif
#ifndef GN_AB_TN16 // A/B: 16 positions per workgroup at every batch size
  if (net.L1 != 128)
    while (tn > (GN_TN_MIN) && (n + tn - 1) / tn < 2048) tn >>= 1;
#endif
  const unsigned tiles = (unsigned)((n + tn - 1) / tn);
  const unsigned grid = swz ? 8 * ((tiles + 7) / 8) : tiles;
  if (net.L1 == 3072) {
    hipLaunchKernelGGL((eval_net_kernel<3072, 1>), dim3(grid), dim3(384), 0, s, net, boards, need, n, out, perm, tiles, swz,
                       rows_out, tn, P, nullptr, nullptr);
  } else if (net.L1 == 128) {
    if (cls)
      hipLaunchKernelGGL((eval_net_kernel<128, 16, true>), dim3(grid), dim3(256), 0, s, net, boards, need, n, out, perm,
                         tiles, swz, rows_out, tn, P, need_small, need_big);
    else
      hipLaunchKernelGGL((eval_net_kernel<128, 16>), dim3(grid), dim3(256), 0, s, net, boards, need, n, out, perm, tiles,
                         swz, rows_out, tn, P, nullptr, nullptr);
  } else if (net.L1 == 1024) {
    hipLaunchKernelGGL((eval_net_kernel<1024, 1>), dim3(grid), dim3(128), 0, s, net, boards, need, n, out, perm, tiles, swz,
                       rows_out, tn, P, nullptr, nullptr);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// -------------------------------------------------------- Eval::evaluate --
__global__ void classify_kernel(const gn_board *__restrict__ boards, size_t n, gn_eval_params P,
                                uint8_t *__restrict__ need_small, uint8_t *__restrict__ need_big) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Board B;
  uint8_t s = 0, b = 0;
  if (unpack(boards[i], B)) {
    const Material m = material(B, P);
    const int us = B.stm;
    const int simple = P.piece_value[0] * (m.pawns[us] - m.pawns[us ^ 1]) + (m.npm[us] - m.npm[us ^ 1]);
    s = abs(simple) > P.small_net_threshold;
    b = !s;
  }
  need_small[i] = s;
  need_big[i] = b;
}

__global__ void reeval_kernel(const int2 *__restrict__ out_small, const uint8_t *__restrict__ need_small, size_t n,
                              gn_eval_params P, uint8_t *__restrict__ need_big) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !need_small[i]) return;
  const int2 o = out_small[i];
  const int32_t nnue = wadd(wmul(P.psqt_weight, o.x), wmul(P.positional_weight, o.y)) / 128;
  if (abs(nnue) < P.reeval_threshold) need_big[i] = 1;
}

__global__ void finalize_kernel(const gn_board *__restrict__ boards, size_t n, int mode,
                                const int2 *__restrict__ out_small, const int2 *__restrict__ out_big,
                                const uint8_t *__restrict__ need_small, const uint8_t *__restrict__ need_big,
                                gn_eval_params P, const Tables *__restrict__ tables, gn_eval *__restrict__ out,
                                const uint32_t *__restrict__ owner, const uint16_t *__restrict__ moves,
                                const Board *__restrict__ unpacked, int score, const uint64_t *__restrict__ counts,
                                NetDevice bnet, const int32_t *__restrict__ part, const int2 *__restrict__ pinfo,
                                uint64_t npos, uint64_t qoff) {
  __shared__ Tables T;
  // (part: the big net's outputs from the sliced stream's partial sums, slice_finish_one --
  // its reads then overlap this kernel's arithmetic instead of running as a kernel of their own)
  __shared__ int4v w1s[8 * 32 * 2];
  if (part) stage_fc1(w1s, bnet);
  load_tables(T, tables);
  // a bounded grid striding over the positions: the 4 KiB table load and its barrier once
  // per workgroup and many positions, not once per 256 (480 k workgroups per expansion)
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
#ifdef GN_AB_FIN_LATE_SUMS // A/B: the sums loaded where the output is needed (after the board)
    auto big_out = [&](size_t j) -> int2 {
      if (part) {
        const int2 info = pinfo[qoff + j];
        if (info.y >= 0) return slice_finish_one<GN_PART_SLICES>(bnet, w1s, part, npos, qoff + j, info);
      }
      return out_big[j];
    };
    const uint32_t ow = unpacked ? owner[i] : 0u;
    const uint16_t mv = unpacked ? moves[i] : (uint16_t)0;
#else
    // the owner and move, then (part) the position's slice sums, all loaded before anything waits:
    // the sums' HBM round trip runs beside the owner -> parent board chain instead of after the
    // board work (owner, parent, pinfo, sums were three round trips in a row)
    const uint32_t ow = unpacked ? owner[i] : 0u;
    const uint16_t mv = unpacked ? moves[i] : (uint16_t)0;
    int2 info = make_int2(0, -1);
    int4v sums[4];
    if (part) {
      info = pinfo[qoff + i];
      // (mode FULL: only the positions the big net evaluates have sums -- the small net's read
      // none; mode BIG: every position, with no load in front of the sums')
      if (mode == GN_MODE_BIG || (mode == GN_MODE_FULL && need_big[i])) slice_sums<GN_PART_SLICES>(part, npos, qoff + i, sums);
    }
    auto big_out = [&](size_t j) -> int2 {
      return part && info.y >= 0 ? slice_finish_from(bnet, w1s, sums, info) : out_big[j];
    };
#endif
    Board B;
    gn_eval e = {0, 0, 0, 0, 0, 0, 0};
    if (unpacked) {
      B = do_move(unpacked[ow], mv, nullptr); // a legal child of a valid parent
    } else if (!unpack(boards[i], B)) {
      e.flags = GN_FLAG_BAD_FEN | GN_FLAG_NO_SCORE;
      out[i] = e;
      continue;
    }
    const Material m = material(B, P);
    bool small;
    int2 o;
    uint32_t flags = 0;
    if (mode == GN_MODE_SMALL) {
      small = true, o = out_small[i];
    } else if (mode == GN_MODE_BIG) {
      small = false, o = big_out(i);
    } else if (need_small[i] && !need_big[i]) {
      small = true, o = out_small[i];
    } else {
      small = false, o = big_out(i);
      if (need_small[i]) flags |= GN_FLAG_REEVAL;
    }
    int32_t nnue = wadd(wmul(P.psqt_weight, o.x), wmul(P.positional_weight, o.y)) / 128;
    const int32_t complexity = abs(wadd(o.x, -o.y));
    nnue = wadd(nnue, -(wmul(nnue, complexity) / (small ? P.complexity_div_small : P.complexity_div_big)));
    const int32_t mat = (small ? P.material_pawn_small : P.material_pawn_big) * (m.pawns[0] + m.pawns[1]) +
                        m.npm[0] + m.npm[1];
    int32_t v = wmul(nnue, P.material_base + mat) / P.material_base;
    v = wadd(v, -(wmul(v, (int32_t)B.rule50) / P.rule50_div));
    v = clampi(v, -P.value_clamp, P.value_clamp);
    if (small) flags |= GN_FLAG_SMALLNET;
    const bool check = in_check(B, T);
    if (check) flags |= GN_FLAG_IN_CHECK;
    e.psqt = o.x, e.positional = o.y, e.final_v = v;
    e.final_cp = wdl_to_cp(v, wdl_material(B, P), P);
    // the score rule's static part (include/gpu_nnue.h); in-check positions with legal moves
    // keep final_cp until score_reduce_kernel replaces it
    if (!score) {
      flags |= GN_FLAG_NO_SCORE; // a child record
    } else if (counts ? counts[i] == 0 : !any_legal(B, T)) {
      flags |= GN_FLAG_NO_MOVES | (check ? GN_FLAG_MATE : 0u); // mate 0 / cp 0
    } else {
      e.score = e.final_cp;
    }
    e.flags = (uint16_t)flags;
    out[i] = e;
  }
}

// ---- the score rule's in-check positions (gpu_nnue.hip resolve_scores) ------------------
// sel[i] = 1 for a scored position in check with a legal move; sel[n] = 0 (the scan's end)
__global__ void score_select_kernel(const gn_eval *__restrict__ out, size_t n, uint64_t *__restrict__ sel) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  uint64_t v = 0;
  if (i < n) {
    const uint32_t f = out[i].flags;
    v = (f & GN_FLAG_IN_CHECK) && !(f & (GN_FLAG_NO_MOVES | GN_FLAG_NO_SCORE | GN_FLAG_BAD_FEN));
  }
  sel[i] = v;
}

// the selected positions, compacted: idx[k] = i, sb[k] = boards[i] for k = pos[i]
__global__ void score_gather_kernel(const gn_board *__restrict__ boards, const uint64_t *__restrict__ sel,
                                    const uint64_t *__restrict__ pos, size_t n, uint32_t *__restrict__ idx,
                                    gn_board *__restrict__ sb) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !sel[i]) return;
  const uint64_t k = pos[i];
  idx[k] = (uint32_t)i;
  sb[k] = boards[i];
}

// An expansion's selected parents (idx) already have every reply evaluated (records rec,
// moves, [off[i], off[i + 1]) per parent i): their reply counts for the compaction's scan ...
__global__ void score_counts_kernel(const uint32_t *__restrict__ idx, size_t m, const uint64_t *__restrict__ off,
                                    uint64_t *__restrict__ counts) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < m) counts[k] = off[idx[k] + 1] - off[idx[k]];
  else if (k == m) counts[m] = 0;
}

// ... and the replies as positions of the rule (compacted at coff[k]): their records with the
// static score part (any legal move? as finalize does for positions), boards and moves.
__global__ void score_replies_kernel(const uint32_t *__restrict__ idx, size_t m, const uint64_t *__restrict__ off,
                                     const uint64_t *__restrict__ coff, const gn_eval *__restrict__ rec,
                                     const uint16_t *__restrict__ moves, const Board *__restrict__ unpacked,
                                     const Tables *__restrict__ tables, gn_eval *__restrict__ ce,
                                     gn_board *__restrict__ cb, uint16_t *__restrict__ cm) {
  __shared__ Tables T;
  load_tables(T, tables);
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  const uint32_t i = idx[k];
  const Board P = unpacked[i];
  uint64_t d = coff[k];
  for (uint64_t c = off[i]; c < off[i + 1]; ++c, ++d) {
    const uint16_t mv = moves[c];
    const Board B = do_move(P, mv, nullptr);
    gn_eval e = rec[c];
    uint32_t f = e.flags & ~GN_FLAG_NO_SCORE;
    e.score = 0;
    if (!any_legal(B, T)) f |= GN_FLAG_NO_MOVES | ((f & GN_FLAG_IN_CHECK) ? GN_FLAG_MATE : 0u);
    else e.score = e.final_cp;
    e.flags = (uint16_t)f;
    ce[d] = e;
    gn_board pb;
    pack(B, pb);
    cb[d] = pb;
    cm[d] = mv;
  }
}

// value = max over the replies c of negate_ply(rule_value(c)) (ties: the smaller move), then
// score / flags / best_move of selected position j; sv (optional) receives the value for
// the level above
__device__ __forceinline__ void score_reduce_one(size_t j, const gn_board *__restrict__ sb, const uint32_t *__restrict__ idx,
                                                 const uint64_t *__restrict__ off, const uint16_t *__restrict__ moves,
                                                 const gn_eval *__restrict__ ce, const int32_t *__restrict__ csv,
                                                 const gn_eval_params &P, gn_eval *__restrict__ out,
                                                 int32_t *__restrict__ sv) {
  // (idx NULL: every position j of sb, those without replies left as they are -- the drop-in's
  // small-batch path, reply_level_kernel, keeps positions in place instead of compacting them)
  if (off[j] == off[j + 1]) return;
  int32_t best = INT32_MIN;
  uint32_t bm = 0xFFFFu;
  for (uint64_t c = off[j]; c < off[j + 1]; ++c) {
    const gn_eval r = ce[c];
    const int32_t v = negate_ply(rule_value(r.flags, r.final_v, csv[c]));
    const uint32_t mv = moves[c];
    if (v > best || (v == best && mv < bm)) best = v, bm = mv;
  }
  Board B;
  unpack(sb[j], B);
  const uint32_t i = idx ? idx[j] : (uint32_t)j;
  gn_eval e = out[i];
  uint32_t fl = (e.flags | GN_FLAG_SEARCHED) & ~GN_FLAG_MATE;
  e.score = rule_score(best, wdl_material(B, P), P, fl);
  e.flags = (uint16_t)fl;
  e.best_move = (uint16_t)bm;
  out[i] = e;
  if (sv) sv[i] = best;
}

__global__ void score_reduce_kernel(const gn_board *__restrict__ sb, size_t m, const uint32_t *__restrict__ idx,
                                    const uint64_t *__restrict__ off, const uint16_t *__restrict__ moves,
                                    const gn_eval *__restrict__ ce, const int32_t *__restrict__ csv,
                                    gn_eval_params P, gn_eval *__restrict__ out, int32_t *__restrict__ sv) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < m) score_reduce_one(j, sb, idx, off, moves, ce, csv, P, out, sv);
}

// Both reductions of the small-batch graph in one workgroup (its two launches, one after the
// other, were ~12 us of a one-game call): level 1's positions (a, their replies' records from
// level 2) and then, after a barrier, level 0's (b, from level 1's records and values the first
// phase wrote -- the same workgroup, so the barrier orders them).
struct ReduceLevel {
  const gn_board *sb;
  size_t m;
  const uint64_t *off;
  const uint16_t *moves;
  const gn_eval *ce;
  const int32_t *csv;
  gn_eval *out;
  int32_t *sv;
};
__global__ void __launch_bounds__(1024) score_reduce2_kernel(ReduceLevel a, ReduceLevel b, gn_eval_params P) {
  for (size_t j = threadIdx.x; j < a.m; j += blockDim.x)
    score_reduce_one(j, a.sb, nullptr, a.off, a.moves, a.ce, a.csv, P, a.out, a.sv);
  __syncthreads();
  for (size_t j = threadIdx.x; j < b.m; j += blockDim.x)
    score_reduce_one(j, b.sb, nullptr, b.off, b.moves, b.ce, b.csv, P, b.out, b.sv);
}

static inline unsigned blocks_for(size_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// Child records for the host (ABI v4 gn_child, include/gpu_nnue.h): psqt, positional and
// final_cp (signed 24 bits) with the low 8 flag bits beside it.  |final_cp| < 2^23 by
// gn_set_eval_params' bound on the win-rate model; the clamp only keeps the field honest.
__global__ void pack_children_kernel(const gn_eval *__restrict__ in, size_t n, gn_child *__restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const gn_eval e = in[i];
  const int32_t cp = clampi(e.final_cp, -(1 << 23) + 1, (1 << 23) - 1);
  gn_child c;
  c.psqt = e.psqt;
  c.positional = e.positional;
  c.cp_flags = (int32_t)(((uint32_t)cp & 0xFFFFFFu) | ((uint32_t)e.flags & 0xFFu) << 24);
  out[i] = c;
}

hipError_t launch_pack_children(const gn_eval *in, size_t n, gn_child *out, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(pack_children_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

hipError_t launch_classify(const gn_board *boards, size_t n, const gn_eval_params &P, uint8_t *need_small,
                           uint8_t *need_big, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(classify_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, boards, n, P, need_small, need_big);
  return hipGetLastError();
}

hipError_t launch_reeval(const int2 *out_small, const uint8_t *need_small, size_t n, const gn_eval_params &P,
                         uint8_t *need_big, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(reeval_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, out_small, need_small, n, P, need_big);
  return hipGetLastError();
}

hipError_t launch_finalize(const gn_board *boards, size_t n, int mode, const int2 *out_small, const int2 *out_big,
                           const uint8_t *need_small, const uint8_t *need_big, const gn_eval_params &P,
                           const Tables *tables, gn_eval *out, hipStream_t s, int score, const uint64_t *counts,
                           const uint32_t *owner, const uint16_t *moves, const Board *unpacked,
                           const SlicedOut *sliced) {
  if (!n) return hipSuccess;
  NetDevice bnet = {};
  if (sliced) bnet = *sliced->net;
  // a bounded grid striding over the positions: each workgroup copies the movegen tables to
  // LDS once (8,192 workgroups: 2.55 -> 2.36 ms per expansion against one per 256 positions)
  constexpr size_t max_blocks = 8192;
  const size_t blocks = std::min<size_t>(blocks_for(n, 256), max_blocks);
  hipLaunchKernelGGL(finalize_kernel, dim3(blocks), dim3(256), 0, s, boards, n, mode, out_small, out_big, need_small,
                     need_big, P, tables, out, owner, moves, unpacked, score, counts, bnet,
                     sliced ? sliced->part : nullptr, sliced ? sliced->pinfo : nullptr, sliced ? sliced->npos : 0,
                     sliced ? sliced->qoff : 0);
  return hipGetLastError();
}

hipError_t launch_score_select(const gn_eval *out, size_t n, uint64_t *sel, hipStream_t s) {
  hipLaunchKernelGGL(score_select_kernel, dim3(blocks_for(n + 1, 256)), dim3(256), 0, s, out, n, sel);
  return hipGetLastError();
}

hipError_t launch_score_gather(const gn_board *boards, const uint64_t *sel, const uint64_t *pos, size_t n,
                               uint32_t *idx, gn_board *sb, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(score_gather_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, boards, sel, pos, n, idx, sb);
  return hipGetLastError();
}

hipError_t launch_score_replies(const uint32_t *idx, size_t m, const uint64_t *off, uint64_t *counts,
                                uint64_t *coff, void *&temp, size_t &temp_bytes, uint64_t *total_host, hipStream_t s) {
  hipError_t e;
  hipLaunchKernelGGL(score_counts_kernel, dim3(blocks_for(m + 1, 256)), dim3(256), 0, s, idx, m, off, counts);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = exclusive_scan_u64(counts, coff, m + 1, temp, temp_bytes, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(total_host, coff + m, sizeof(uint64_t), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  return hipStreamSynchronize(s);
}

hipError_t launch_score_replies_fill(const uint32_t *idx, size_t m, const uint64_t *off, const uint64_t *coff,
                                     const gn_eval *rec, const uint16_t *moves, const Board *unpacked,
                                     const Tables *tables, gn_eval *ce, gn_board *cb, uint16_t *cm, hipStream_t s) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(score_replies_kernel, dim3(blocks_for(m, 256)), dim3(256), 0, s, idx, m, off, coff, rec, moves,
                     unpacked, tables, ce, cb, cm);
  return hipGetLastError();
}

// One level of the score rule's replies for a small batch (the drop-in's gn_evaluate_batch,
// gpu_nnue.hip FastBatch), as one workgroup and no host round trip: position i of boards is
// selected as score_select_kernel selects its record -- a valid board, in check, with a legal
// move (every position of the graph is a scored one) -- from the board alone, so that the levels
// need no evaluation before them; off[i] = the
// exclusive prefix of the selected positions' legal-move counts (off[n] = their total; both
// clamped to cap); the
// replies, in gen_legal order, are rb / rm [off[i], off[i + 1]) -- the boards write_children
// would make -- and every slot from the total to cap is an empty board (an invalid position for
// the evaluation that follows, so that launches sized by cap need no count).  A total beyond cap
// sets *flag (the caller then takes the general path); first: *flag is set, else or'd.
// GN_RL_THREADS threads (a 1,024-thread version spilled 35 VGPRs around gen_legal and took 36 us per
// launch); positions per thread <= 16,384 / threads (n <= 16,384: level 2 takes level 1's capacity).
// One move generation per position: a thread keeps its positions' legal moves (and which of its
// positions each belongs to) in its LDS segment of MAXM entries, and after the scan every thread
// makes the replies r = t, t + NT, ... -- the thread owning r by a binary search over the scan --
// so that a position's ~30 do_move + pack run on 30 lanes, not one after another on one.  (Two
// move generations and a serial write per in-check position took 40 us per launch, the drop-in's
// largest kernel.)  A thread whose replies overflow its segment writes them itself, as before.
// reply_level_kernel's workgroup: 512 threads (two positions per thread at the 1,024-position
// class): p50 0.135 -> 0.130 ms, 16 coalesced callers 2.8 -> 3.15 M positions/s against 256
// (round 6, profiles/r06/dropin_ab_r06x.txt); the LDS segments hold 16,384 moves either way
#ifndef GN_RL_THREADS
#define GN_RL_THREADS 512
#endif
__global__ void __launch_bounds__(GN_RL_THREADS) reply_level_kernel(const gn_board *__restrict__ boards, uint32_t n,
                                                           const Tables *__restrict__ tables, uint64_t *__restrict__ off,
                                                           uint32_t cap, gn_board *__restrict__ rb,
                                                           uint16_t *__restrict__ rm, uint32_t *__restrict__ flag,
                                                           int first) {
  constexpr uint32_t NT = GN_RL_THREADS, MAXM = 16384 / NT;
  __shared__ Tables T;
  __shared__ uint32_t part[NT];
  __shared__ uint16_t smv[NT][MAXM]; // a thread's replies' moves ...
  __shared__ uint8_t spos[NT][MAXM]; // ... and their positions (offsets from the thread's first)
  load_tables(T, tables);
  const uint32_t t = threadIdx.x, q = (n + NT - 1) / NT, lo = t * q, hi = lo + q < n ? lo + q : n;
  uint32_t c = 0;
#pragma unroll 1
  for (uint32_t i = lo; i < hi; ++i) {
    uint32_t cnt = 0;
    Board B;
    if (unpack(boards[i], B) && in_check(B, T))
      gen_legal(B, T, [&](uint16_t m) {
        if (c + cnt < MAXM) smv[t][c + cnt] = m, spos[t][c + cnt] = (uint8_t)(i - lo);
        ++cnt;
      });
    off[i] = cnt;
    c += cnt;
  }
  part[t] = c;
  __syncthreads();
  for (uint32_t d = 1; d < NT; d <<= 1) { // inclusive scan of the per-thread totals (Hillis-Steele)
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const uint32_t total = part[NT - 1];
  uint32_t base = part[t] - c;
  const bool spill = c > MAXM;
#pragma unroll 1
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t cnt = (uint32_t)off[i];
    // (offsets clamped to cap: past an overflow every position's range stays inside the reply
    // buffers, so the launches after this one -- sized by cap, the call then rerun on the general
    // path -- never read past them; unclamped, score_reduce_kernel read up to the uncapped total and
    // faulted, round 6)
    off[i] = base < cap ? base : cap;
    if (spill && cnt) { // this thread's replies did not fit its segment: made here, in order
      Board B;
      unpack(boards[i], B);
      uint32_t r = base;
      gen_legal(B, T, [&](uint16_t m) {
        if (r < cap) {
          pack(do_move(B, m, nullptr), rb[r]);
          rm[r] = m;
        }
        ++r;
      });
    }
    base += cnt;
  }
  const uint32_t lim = total < cap ? total : cap;
#pragma unroll 1
  for (uint32_t r = t; r < lim; r += NT) {
    uint32_t u = 0; // the first thread u with part[u] > r (part: inclusive, nondecreasing)
#pragma unroll
    for (uint32_t step = NT / 2; step; step >>= 1)
      if (part[u + step - 1] <= r) u += step;
    const uint32_t cu = part[u] - (u ? part[u - 1] : 0u);
    if (cu > MAXM) continue; // (a spilled thread's, written above)
    const uint32_t k = r - (part[u] - cu);
    const uint16_t m = smv[u][k];
    Board B;
    unpack(boards[u * q + spos[u][k]], B);
    pack(do_move(B, m, nullptr), rb[r]);
    rm[r] = m;
  }
  if (t == 0) {
    off[n] = total < cap ? total : cap;
    if (first) *flag = total > cap ? 1u : 0u;
    else if (total > cap) atomicOr(flag, 1u);
  }
  for (uint32_t r = total + t; r < cap; r += NT) rb[r] = gn_board{};
}

hipError_t launch_reply_level(const gn_board *boards, size_t n, const Tables *tables, uint64_t *off, size_t cap,
                              gn_board *rb, uint16_t *rm, uint32_t *flag, int first, hipStream_t s) {
  if (!n || n > 16384 || cap >= 0x80000000ull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(reply_level_kernel, dim3(1), dim3(GN_RL_THREADS), 0, s, boards, (uint32_t)n, tables, off,
                     (uint32_t)cap, rb, rm, flag, first);
  return hipGetLastError();
}

hipError_t launch_score_reduce2(const gn_board *sb1, size_t m1, const uint64_t *off1, const uint16_t *moves2,
                                const gn_eval *ce2, const int32_t *csv2, gn_eval *out1, int32_t *sv1,
                                const gn_board *sb0, size_t m0, const uint64_t *off0, const uint16_t *moves1,
                                const gn_eval_params &P, gn_eval *out0, hipStream_t s) {
  const ReduceLevel a = {sb1, m1, off1, moves2, ce2, csv2, out1, sv1}, b = {sb0, m0, off0, moves1, out1, sv1, out0, nullptr};
  hipLaunchKernelGGL(score_reduce2_kernel, dim3(1), dim3(1024), 0, s, a, b, P);
  return hipGetLastError();
}

hipError_t launch_score_reduce(const gn_board *sb, size_t m, const uint32_t *idx, const uint64_t *off,
                               const uint16_t *moves, const gn_eval *ce, const int32_t *csv, const gn_eval_params &P,
                               gn_eval *out, int32_t *sv, hipStream_t s) {
  if (!m) return hipSuccess;
  hipLaunchKernelGGL(score_reduce_kernel, dim3(blocks_for(m, 256)), dim3(256), 0, s, sb, m, idx, off, moves, ce, csv,
                     P, out, sv);
  return hipGetLastError();
}

// ------------------------------------------------------- movegen kernels --
__global__ void count_children_kernel(const gn_board *__restrict__ boards, size_t n, const Tables *__restrict__ tables,
                                      uint64_t *__restrict__ counts, uint64_t *__restrict__ ebound) {
  __shared__ Tables T;
  load_tables(T, tables);
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Board B;
  uint64_t c = 0, kmoves = 0;
  if (unpack(boards[i], B)) {
    const Bitboard king = B.byType[KING] & color_bb(B, B.stm);
    gen_legal(B, T, [&](uint16_t m) {
      ++c;
      kmoves += (sqbb(move_from(m)) & king) != 0;
    });
  }
  counts[i] = c;
  if (ebound) { // planned-expansion entries of this parent (stream.hip), bounded: its refresh
    // (bias + P rows + the cache store per list, or the cache row + <= P differences + the
    // store) or its carry entries, after <= GN_SCR_GAP no-ops per list; per child
    // <= 4 delta entries per list, or for a king move a refresh (bias + <= P rows + the
    // cache store, after <= GN_SCR_GAP no-ops) + the other perspective's <= 4; per-tile
    // padding (<= 3 per list per tile the parent touches)
    const uint64_t P = popcnt(B.byType[0]);
    ebound[i] = c || P ? 2 * (P + 2) + 2 * GN_SCR_GAP + 8 * (c - kmoves) + (P + 6 + GN_SCR_GAP) * kmoves +
                             6 * ((c + 1) / 16 + 2)
                       : 0;
  }
}

// Children in two passes: child_moves_kernel (a thread per parent) lists the legal moves,
// the owning parent of every child and the chained-walk link; child_boards_kernel (a thread
// per child) makes the child and its feature-transformer delta.  A thread per parent
// writing ~31 children of 58 B each left partial L2 lines to be written back (4.5x the
// bytes); a thread per child writes every array coalesced.
//
// The link, next_slot[i]: the child whose placement is boards[i + 1]'s (a game's next
// position; no two legal moves give one placement); the chained walk then starts parent
// i + 1 from that child's accumulators, gathering one carry row per perspective instead
// of its refresh.  Found per parent without making any child: S is the set of squares on
// which the parent's and the next board's placements differ; a move can give the next
// placement only when the squares it changes are exactly S, the occupancy it leaves is the
// next board's and the piece(s) it puts down stand there in the next board -- then the two
// placements agree on every square.  (Packing each child to compare it cost the per-child
// pass 3.1 ms a step of its 5.8: every wave held a linked lane.)
__global__ void child_moves_kernel(const gn_board *__restrict__ boards, size_t n, const Tables *__restrict__ tables,
                                   const uint64_t *__restrict__ offsets, uint16_t *__restrict__ moves,
                                   uint32_t *__restrict__ owner, uint8_t *__restrict__ next_slot, int chain_k,
                                   unsigned long long *__restrict__ rows, Board *__restrict__ unpacked) {
  __shared__ Tables T;
  load_tables(T, tables);
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t slot = 255;
  Board B;
  if (!unpack(boards[i], B)) {
    if (next_slot) next_slot[i] = 255;
    return;
  }
  if (unpacked) unpacked[i] = B; // for child_boards_kernel (a valid board has children only)
  // S (0: no link possible) and the next board's bitboards
  Board N;
  Bitboard S = 0;
  if (next_slot && i + 1 < n) {
    const gn_board nb = boards[i + 1];
    const int pn = popcnt(nb.occ);
    if (pn >= 2 && pn <= 32) { // a child has 2..32 pieces
      unpack(nb, N);           // a bad piece nibble leaves its square out of N's types: in S
      S = (B.byColor[0] ^ N.byColor[0]) | (B.byColor[1] ^ N.byColor[1]) | (B.byType[0] ^ N.byType[0]);
#pragma unroll
      for (int t = PAWN; t <= KING; ++t) S |= B.byType[t] ^ N.byType[t];
    }
  }
  const int us = B.stm;
  const Bitboard occ = B.byType[0];
  const uint64_t k0 = offsets[i];
  uint64_t k = k0;
  gen_legal(B, T, [&](uint16_t m) {
    moves[k] = m;
    owner[k] = (uint32_t)i;
    if (S) {
      const int from = move_from(m), to = move_to(m), type = move_type(m);
      Bitboard sm, cocc;
      int kto = to, rto = to;
      if (type == MT_CASTLING) {
        const int kside = to > from;
        kto = rel_sq(us, kside ? 6 : 2), rto = rel_sq(us, kside ? 5 : 3);
        sm = (kto != from ? sqbb(from) | sqbb(kto) : 0) | (rto != to ? sqbb(to) | sqbb(rto) : 0);
        cocc = (occ ^ sqbb(from) ^ sqbb(to)) | sqbb(kto) | sqbb(rto);
      } else {
        const int capsq = type == MT_EN_PASSANT ? to - (us == WHITE ? 8 : -8) : to;
        sm = sqbb(from) | sqbb(to) | sqbb(capsq);
        cocc = (occ & ~(sqbb(from) | sqbb(capsq))) | sqbb(to);
      }
      if (sm == S && cocc == N.byType[0]) { // the pieces put down
        bool same;
        if (type == MT_CASTLING)
          same = (N.byType[KING] & N.byColor[us] & sqbb(kto)) && (N.byType[ROOK] & N.byColor[us] & sqbb(rto));
        else
          same = piece_on(N, to) ==
                 (type == MT_PROMOTION ? make_piece(us, move_promo(m)) : piece_on(B, from));
        if (same) slot = (uint32_t)(k - k0);
      }
    }
    ++k;
  });
  if (next_slot) next_slot[i] = (uint8_t)slot;
  // feature-transformer rows the incremental evaluation will gather: the parent's
  // refresh (both perspectives) here -- or, for a linked next board of the same chain,
  // one carry row per perspective instead of that board's refresh -- each child's in
  // child_boards_kernel
  if (rows) {
    unsigned long long r = 2ull * popcnt(occ);
    if (slot != 255 && chain_k > 1 && (i + 1) % (size_t)chain_k != 0) r -= 2ull * popcnt(N.byType[0]) - 2;
    atomicAdd(rows, r); // modulo 2^64: the sum over all threads is the count
  }
}

__global__ void child_boards_kernel(const gn_board *__restrict__ boards, size_t c0, size_t nc,
                                    const uint16_t *__restrict__ moves, const uint32_t *__restrict__ owner,
                                    gn_board *__restrict__ children, ChildDelta *__restrict__ deltas,
                                    unsigned long long *__restrict__ rows, const Board *__restrict__ unpacked) {
  const size_t c = c0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long nr = 0;
  if (c < c0 + nc) {
    const uint32_t i = owner[c];
    Board B;
    if (unpacked) B = unpacked[i]; // the siblings share it (one cache line run per parent)
    else unpack(boards[i], B);     // valid: an invalid parent has no children
    Dirty d;
    const Board C = do_move(B, moves[c], &d);
    if (children) pack(C, children[c]); // stored when the caller keeps the boards
    if (deltas) deltas[c] = make_child_delta(B, C, d);
    // per child either the delta rows or a refresh of the perspective whose king moved
    nr = d.king_moved ? popcnt(C.byType[0]) + d.n_rem + d.n_add : 2 * (d.n_rem + d.n_add);
  }
  if (rows) { // one atomic per workgroup
    __shared__ unsigned long long part[GN_FRONT_WG / 64];
#pragma unroll
    for (int off = 32; off; off >>= 1) nr += __shfl_down(nr, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = nr;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long t = 0;
#pragma unroll
      for (int w = 0; w < GN_FRONT_WG / 64; ++w) t += part[w];
      atomicAdd(rows, t);
    }
  }
}

__global__ void count_sum_kernel(const gn_board *__restrict__ boards, size_t n, const Tables *__restrict__ tables,
                                 unsigned long long *__restrict__ total) {
  __shared__ Tables T;
  __shared__ unsigned long long part[4];
  load_tables(T, tables);
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c = 0;
  if (i < n) {
    Board B;
    if (unpack(boards[i], B)) gen_legal(B, T, [&](uint16_t) { ++c; });
  }
  for (int off = 32; off; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += part[w];
    if (s) atomicAdd(total, s);
  }
}

__global__ void random_positions_kernel(uint64_t seed, size_t first, size_t n, int max_plies,
                                        const Tables *__restrict__ tables, gn_board *__restrict__ out) {
  __shared__ Tables T;
  load_tables(T, tables);
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gn_board pb;
  pack(random_playout(seed + first + i, max_plies, T), pb);
  out[i] = pb;
}

__global__ void random_games_kernel(uint64_t seed, size_t first_game, size_t n_games, int plies,
                                    const Tables *__restrict__ tables, gn_board *__restrict__ out) {
  __shared__ Tables T;
  load_tables(T, tables);
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_games) return;
  gn_board *dst = out + g * (size_t)(plies + 1);
  random_game(seed + first_game + g, plies, T, [&](int k, const Board &B, uint16_t) {
    gn_board pb;
    pack(B, pb);
    dst[k] = pb;
  });
}

// Lichess batches replayed on the GPU (gn_evaluate_games; IncomingBatch::from_acquired,
// /root/reference/src/queue.rs:548-700): one thread per game resolves the game's move codes
// (uci_code) one after another with resolve_uci (shakmaty's UciMove::to_move rule) and writes
// position k (the root after k moves) to boards[moff[g] + g + k] and the resolved move to
// smoves[moff[g] + k - 1]; status[g] = 0, or k for the first move k (1-based) that is not
// legal (the game then fails, as `uci.to_move(&pos)?` fails the batch, queue.rs:576).
__global__ void replay_games_kernel(const gn_board *__restrict__ roots, size_t ng, const uint64_t *__restrict__ moff,
                                    const uint16_t *__restrict__ codes, const Tables *__restrict__ tables,
                                    gn_board *__restrict__ boards, uint16_t *__restrict__ smoves,
                                    int32_t *__restrict__ status) {
  __shared__ Tables T;
  load_tables(T, tables);
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ng) return;
  const uint64_t m0 = moff[g], m1 = moff[g + 1];
  gn_board *dst = boards + m0 + g;
  Board B;
  unpack(roots[g], B); // validated by the host's FEN parser
  dst[0] = roots[g];
  int32_t st = 0;
  for (uint64_t k = m0; k < m1; ++k) {
    uint16_t mv = 0;
    if (!resolve_uci(B, T, codes[k], mv)) {
      st = (int32_t)(k - m0) + 1;
      break;
    }
    B = do_move(B, mv, nullptr);
    gn_board pb;
    pack(B, pb);
    dst[k - m0 + 1] = pb;
    smoves[k] = mv;
  }
  status[g] = st;
}

__global__ void gather_boards_kernel(const gn_board *__restrict__ src, const uint32_t *__restrict__ idx, size_t n,
                                     gn_board *__restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

// sort key of a position: both king squares (L2 locality of the king-bucket slices),
// then one bit per home square (ranks 1, 2, 7, 8 without e1 / e8, in square order):
// the start position's piece still stands there.  A tile of 16 positions then shares
// its kings and unmoved pieces (eval_net's common-row base); invalid last.
// Key = uint16_t: kings only (wk << 6 | bk), for small-net-only batches.
// bkt: the layer-stack bucket ((pieces - 1) / 4) enters the key, so that a tile's 16
// positions mostly share one bucket and the layer stack runs once per tile instead of
// once per bucket present: small net above the kings (its table is L2-resident, the king
// order buys little there), big net between the kings and the home-square bits.
template <class Key>
__global__ void king_keys_kernel(const gn_board *__restrict__ boards, size_t n, Key *__restrict__ keys,
                                 uint32_t *__restrict__ idx, int bkt) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const gn_board p = boards[i];
  uint64_t wlo, whi;
  piece_words(p, wlo, whi);
  uint64_t o = p.occ;
  int wk = 64, bk = 64;
  uint64_t home = 0; // bit s: square s holds its start-position piece
  const int c = popcnt(o) <= 32 ? popcnt(o) : 0;
  for (int k = 0; k < c; ++k) {
    const int s = pop_lsb(o), pc = piece_nibble(wlo, whi, k);
    if (pc == make_piece(WHITE, KING)) wk = s;
    if (pc == make_piece(BLACK, KING)) bk = s;
    const int r = s >> 3, f = s & 7;
    constexpr int BACK[8] = {ROOK, KNIGHT, BISHOP, QUEEN, KING, BISHOP, KNIGHT, ROOK};
    const int want = r == 0 ? make_piece(WHITE, BACK[f]) : r == 1 ? make_piece(WHITE, PAWN)
                   : r == 6 ? make_piece(BLACK, PAWN) : r == 7 ? make_piece(BLACK, BACK[f]) : -1;
    if (pc == want) home |= 1ull << s;
  }
  const uint32_t b = c ? (uint32_t)(c - 1) / 4 : 0;
  if constexpr (sizeof(Key) == 2) {
    keys[i] = (Key)(wk < 64 && bk < 64 ? ((bkt ? b << 12 : 0u) | (uint32_t)(wk << 6 | bk)) : 0xFFFF);
    idx[i] = (uint32_t)i;
    return;
  }
  uint64_t key = ~0ull;
  if (wk < 64 && bk < 64) {
    // 30 home squares: a1-d1, f1-h1, rank 2, rank 7, a8-d8, f8-h8 -> bits 51..22
    const uint64_t lo16 = home & 0xFFFF, hi16 = home >> 48;
    const uint64_t h30 = (lo16 & 0xF) | ((lo16 >> 1) & ~0xFull) // 15 bits: squares 0-3, 5-15
                         | ((hi16 & 0xFFF) | ((hi16 >> 1) & ~0xFFFull)) << 15; // 15 bits: 48-59, 61-63
    uint64_t r = 0, t = h30; // square order, lowest square most significant
    for (int k = 0; k < 30; ++k, t >>= 1) r = r << 1 | (t & 1);
    key = bkt ? (uint64_t)wk << 58 | (uint64_t)bk << 52 | (uint64_t)b << 49 | r << 19
              : (uint64_t)wk << 58 | (uint64_t)bk << 52 | r << 22;
  }
  keys[i] = (Key)key;
  idx[i] = (uint32_t)i;
}

// Position-sensitive 64-bit checksum of a device buffer: sum over 8-byte words w_i of
// splitmix64(w_i ^ (i * golden)) (wrapping), so equal buffers give equal sums and a
// moved or changed word changes it.  Tail bytes are zero-padded into a last word.
__global__ void checksum_kernel(const uint8_t *__restrict__ p, size_t bytes, unsigned long long *__restrict__ out) {
  const size_t nw = (bytes + 7) / 8;
  unsigned long long acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t w = 0;
    if (8 * i + 8 <= bytes) w = *reinterpret_cast<const uint64_t *>(p + 8 * i);
    else
      for (size_t k = 8 * i; k < bytes; ++k) w |= (uint64_t)p[k] << (8 * (k - 8 * i));
    acc += Xoshiro::mix(w ^ (i * 0x9E3779B97F4A7C15ull));
  }
  for (int off = 32; off; off >>= 1) acc += __shfl_down(acc, off, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

hipError_t launch_checksum(const void *p, size_t bytes, unsigned long long *out, hipStream_t s) {
  if (!bytes) return hipSuccess;
  const size_t nw = (bytes + 7) / 8;
  const unsigned g = (unsigned)std::min<size_t>(8192, (nw + 255) / 256);
  hipLaunchKernelGGL(checksum_kernel, dim3(g), dim3(256), 0, s, (const uint8_t *)p, bytes, out);
  return hipGetLastError();
}

__global__ void offsets_u32_kernel(const uint64_t *__restrict__ in, size_t n, uint32_t *__restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (uint32_t)in[i];
}

hipError_t launch_count_children(const gn_board *boards, size_t n, const Tables *tables, uint64_t *counts,
                                 hipStream_t s, uint64_t *ebound) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(count_children_kernel, dim3(blocks_for(n, GN_FRONT_WG)), dim3(GN_FRONT_WG), 0, s, boards, n, tables, counts,
                     ebound);
  return hipGetLastError();
}

hipError_t launch_write_children(const gn_board *boards, size_t n, const Tables *tables, const uint64_t *offsets,
                                 size_t c0, size_t nc, gn_board *children, uint16_t *moves, uint32_t *owner,
                                 ChildDelta *deltas, uint8_t *next_slot, int chain_k, unsigned long long *rows,
                                 hipStream_t s, Board *unpacked) {
  if (!n) return hipSuccess;
  if (!moves || !owner) return hipErrorInvalidValue;
  hipLaunchKernelGGL(child_moves_kernel, dim3(blocks_for(n, GN_FRONT_WG)), dim3(GN_FRONT_WG), 0, s, boards, n, tables, offsets, moves,
                     owner, next_slot, chain_k, rows, unpacked);
  if (nc)
    hipLaunchKernelGGL(child_boards_kernel, dim3(blocks_for(nc, GN_FRONT_WG)), dim3(GN_FRONT_WG), 0, s, boards, c0, nc, moves, owner,
                       children, deltas, rows, unpacked);
  return hipGetLastError();
}

hipError_t launch_count_sum(const gn_board *boards, size_t n, const Tables *tables, unsigned long long *total,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(count_sum_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, boards, n, tables, total);
  return hipGetLastError();
}

hipError_t launch_random_positions(uint64_t seed, size_t first, size_t n, int max_plies, const Tables *tables,
                                   gn_board *out, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(random_positions_kernel, dim3(blocks_for(n, 128)), dim3(128), 0, s, seed, first, n, max_plies,
                     tables, out);
  return hipGetLastError();
}

hipError_t launch_random_games(uint64_t seed, size_t first_game, size_t n_games, int plies, const Tables *tables,
                               gn_board *out, hipStream_t s) {
  if (!n_games) return hipSuccess;
  hipLaunchKernelGGL(random_games_kernel, dim3(blocks_for(n_games, 128)), dim3(128), 0, s, seed, first_game, n_games,
                     plies, tables, out);
  return hipGetLastError();
}

hipError_t launch_replay_games(const gn_board *roots, size_t ng, const uint64_t *moff, const uint16_t *codes,
                               const Tables *tables, gn_board *boards, uint16_t *smoves, int32_t *status, hipStream_t s) {
  if (!ng) return hipSuccess;
  hipLaunchKernelGGL(replay_games_kernel, dim3(blocks_for(ng, 64)), dim3(64), 0, s, roots, ng, moff, codes, tables,
                     boards, smoves, status);
  return hipGetLastError();
}

hipError_t launch_gather_boards(const gn_board *src, const uint32_t *idx, size_t n, gn_board *dst, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(gather_boards_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, src, idx, n, dst);
  return hipGetLastError();
}

hipError_t launch_offsets_u32(const uint64_t *in, size_t n, uint32_t *out, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(offsets_u32_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

template <class Key>
static hipError_t king_sort_t(const gn_board *boards, size_t n, Key *keys, uint32_t *idx, Key *keys_out,
                              uint32_t *perm, void *&temp, size_t &temp_bytes, hipStream_t s) {
  constexpr int bkt = 1; // the layer-stack bucket in the key (king_keys_kernel)
  hipLaunchKernelGGL(king_keys_kernel<Key>, dim3(blocks_for(n, 256)), dim3(256), 0, s, boards, n, keys, idx, bkt);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  constexpr int BITS = 8 * sizeof(Key);
  size_t need = 0;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, need, keys, keys_out, idx, perm, (int)n, 0, BITS, s);
  if (e != hipSuccess) return e;
  if (need > temp_bytes) {
    if (temp) (void)hipFree(temp);
    temp = nullptr;
    temp_bytes = 0;
    if ((e = hipMalloc(&temp, need)) != hipSuccess) return e;
    temp_bytes = need;
  }
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys, keys_out, idx, perm, (int)n, 0, BITS, s);
}

hipError_t king_sort(const gn_board *boards, size_t n, uint64_t *keys, uint32_t *idx, uint64_t *keys_out,
                     uint32_t *perm, bool placement, void *&temp, size_t &temp_bytes, hipStream_t s) {
  if (!n) return hipSuccess;
  if (placement) return king_sort_t(boards, n, keys, idx, keys_out, perm, temp, temp_bytes, s);
  return king_sort_t(boards, n, reinterpret_cast<uint16_t *>(keys), idx, reinterpret_cast<uint16_t *>(keys_out), perm,
                     temp, temp_bytes, s);
}

// Block order of the planned expansion (stream_eval_kernel's order[]): blocks sorted by
// the king squares of their middle parent, so that the blocks an XCD runs together (the
// XCD swizzle gives it a contiguous eighth of this order) gather from the same king-bucket
// slices of the FT and share the XCD's L2.  keys: uint16 (wk << 6 | bk; 4095: invalid).
__global__ void block_keys_kernel(const gn_board *__restrict__ parents, size_t n, uint32_t K, uint32_t nblk,
                                  uint16_t *__restrict__ keys, uint32_t *__restrict__ idx) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblk) return;
  const size_t pb = (size_t)b * K, pe = pb + K < n ? pb + K : n;
  // the block's middle parent keys it (first / quarter / three-quarter parents and Morton or
  // black-king-major orders of the king squares or buckets all measured within +-0.5 %)
  const gn_board p = parents[pb + (pe - pb) / 2];
  uint64_t wlo, whi;
  piece_words(p, wlo, whi);
  uint64_t o = p.occ;
  int wk = 63, bk = 63;
  const int c = popcnt(o) <= 32 ? popcnt(o) : 0;
  for (int k = 0; k < c; ++k) {
    const int sq = pop_lsb(o), pc = piece_nibble(wlo, whi, k);
    if (pc == make_piece(WHITE, KING)) wk = sq;
    if (pc == make_piece(BLACK, KING)) bk = sq;
  }
  keys[b] = (uint16_t)(wk << 6 | bk);
  idx[b] = b;
}

hipError_t block_order(const gn_board *parents, size_t n, uint32_t K, uint32_t nblk, uint16_t *keys, uint32_t *idx,
                       uint16_t *keys_out, uint32_t *order, void *&temp, size_t &temp_bytes, hipStream_t s) {
  if (!nblk) return hipSuccess;
  hipLaunchKernelGGL(block_keys_kernel, dim3(blocks_for(nblk, GN_FRONT_WG)), dim3(GN_FRONT_WG), 0, s, parents, n, K, nblk, keys, idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t need = 0;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, need, keys, keys_out, idx, order, (int)nblk, 0, 12, s);
  if (e != hipSuccess) return e;
  if (need > temp_bytes) {
    if (temp) (void)hipFree(temp);
    temp = nullptr;
    temp_bytes = 0;
    if ((e = hipMalloc(&temp, need)) != hipSuccess) return e;
    temp_bytes = need;
  }
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys, keys_out, idx, order, (int)nblk, 0, 12, s);
}

hipError_t exclusive_scan_u64(const uint64_t *counts, uint64_t *offsets, size_t n1, void *&temp, size_t &temp_bytes,
                              hipStream_t s) {
  size_t need = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need, counts, offsets, n1, s);
  if (e != hipSuccess) return e;
  if (need > temp_bytes) {
    if (temp) (void)hipFree(temp);
    temp = nullptr;
    temp_bytes = 0;
    if ((e = hipMalloc(&temp, need)) != hipSuccess) return e;
    temp_bytes = need;
  }
  return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, counts, offsets, n1, s);
}

hipError_t launch_expand_net(const NetDevice &net, const gn_board *parents, size_t n, const uint64_t *offsets,
                             const gn_board *children, const ChildDelta *deltas, const uint8_t *need_parent,
                             const uint8_t *need_child, int2 *out_parent, int2 *out_child, int swz, hipStream_t s) {
  if (!n) return hipSuccess;
  if (n >= 0x80000000ull) return hipErrorInvalidValue; // 32-bit parent indices in the kernels
  // the big nets (L1 3072 / 1024) always run planned (stream.hip, launch_plan_stream)
  if (net.L1 != 128) return hipErrorInvalidValue;
  const unsigned g = (unsigned)(swz ? 8 * ((n + 7) / 8) : n);
  hipLaunchKernelGGL((expand_eval_kernel<128, 16>), dim3(g), dim3(256), 0, s, net, parents, offsets, children, deltas,
                     need_parent, need_child, out_parent, out_child, n, swz);
  return hipGetLastError();
}

} // namespace gn
