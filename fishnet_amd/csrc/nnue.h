// nnue.h — Stockfish NNUE (HalfKAv2_hm, SF 17.1-era) as laid out in HBM by
// libgpu_nnue, shared between the host loader and the kernels.
//
// HBM layout of one network (all arrays 256-B aligned):
//   ft      [22528][RS] bytes, RS = 2*L1 + 32: one feature's row is the L1
//           int16 feature-transformer weights (doubled at load, as Stockfish
//           scale_weights does) followed by its 8 int32 PSQT weights, so one
//           gathered feature = one contiguous row (6,176 B big / 288 B small)
//   bias    [L1] int16 (doubled)
//   w0      [8 buckets][16][L1] int8     b0 [8][16] int32    (fc_0)
//   w1      [8][32][32] int8             b1 [8][32] int32    (fc_1, cols 30,31 pad)
//   w2      [8][32] int8                 b2 [8] int32        (fc_2)
#pragma once
#include <stdint.h>

#include "chess.h"

namespace gn {

constexpr int FT_INPUTS = 22528;
constexpr int PSQT_BUCKETS = 8;
constexpr int LAYER_STACKS = 8;
constexpr uint32_t NNUE_VERSION = 0x7AF32F20u;

struct NetDevice {
  int L1;
  uint32_t row_stride;
  const uint8_t *ft;
  const int16_t *bias;
  const int8_t *w0;
  const int32_t *b0;
  const int8_t *w1;
  const int32_t *b1;
  const int8_t *w2;
  const int32_t *b2;
};

// HalfKAv2_hm feature index:
//   (sq ^ orient) + 64 * plane(piece, perspective) + 704 * king_bucket
// orient mirrors files when the perspective's king is on files a-d and flips
// ranks for black; king_bucket = 4 * (7 - relative rank) + min(file, 7 - file);
// planes: own P N B R Q = 0 2 4 6 8, their P N B R Q = 1 3 5 7 9, kings = 10.
GN_HD int feature_index(int persp, int sq, int pc, int ksq) {
  const int kf = ksq & 7;
  const int orient = (kf < 4 ? 7 : 0) ^ (persp ? 56 : 0);
  const int rel_rank = (ksq >> 3) ^ (persp ? 7 : 0);
  const int bucket = 4 * (7 - rel_rank) + (kf < 4 ? kf : 7 - kf);
  const int pt = pc & 7;
  const int plane = pt == KING ? 10 : 2 * (pt - 1) + ((pc >> 3) != persp);
  return (sq ^ orient) + 64 * plane + 704 * bucket;
}

// 32-bit hashes stored in .nnue files
inline uint32_t affine_hash(uint32_t prev, uint32_t outs) {
  uint32_t h = 0xCC03DAE4u + outs;
  h ^= prev >> 1;
  h ^= prev << 31;
  return h;
}
inline uint32_t ft_hash(int l1) { return 0x7f234cb8u ^ (uint32_t)(l1 * 2); }
inline uint32_t arch_hash(int l1) {
  uint32_t h = 0xEC42E90Du ^ (uint32_t)(l1 * 2);
  h = affine_hash(h, 16);
  h = 0x538D24C7u + h;
  h = affine_hash(h, 32);
  h = 0x538D24C7u + h;
  return affine_hash(h, 1);
}

} // namespace gn
