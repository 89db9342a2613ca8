// f32-accurate contractions on the bf16 matrix cores.
//
// gfx950 runs v_mfma_f32_16x16x32_bf16 at 16x the FLOP rate of the f32-input
// v_mfma_f32_16x16x4_f32.  Every f32 operand is split EXACTLY into three bf16
// pieces by truncation, x = h + m + l (h keeps the top 8 significand bits, the
// residual x - h has <= 16 bits, m its top 8, and l the last <= 8 bits, so
// each subtraction is exact and l is representable).  Products of bf16 pieces
// are exact in the f32 accumulator, so
//   * uint8-valued operand (pixels, exact in bf16) x f32: 3 MFMAs
//     (A.l + A.m summed first into a "small" accumulator, A.h into a "big" one);
//   * f32 x f32: the 6 terms whose weight is >= 2^-16 (hh | hm, mh, hl, mm, lh);
//     the 3 dropped terms are <= 2^-24 |a b| each.
// Measured on MI355X (scripts/mfma_numerics.hip, K = 256, 50 random tiles):
// max |err| / sum|a b| = 5.0e-8 (uint8 x f32) and 6.1e-8 (f32 x f32) with the
// big / small accumulator split, against 1.8e-7 / 1.9e-7 for the exact-f32
// v_mfma_f32_16x16x4_f32 k-ordered fma chain.  Tests hold these paths to the
// same tolerances as the f32 ones.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));

// exact split x = h + m + l; returns the three bf16 bit patterns in the low 16 bits
__device__ inline void split3(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
  const uint32_t hb = __float_as_uint(x) & 0xffff0000u;
  const float r1 = __fsub_rn(x, __uint_as_float(hb));
  const uint32_t mb = __float_as_uint(r1) & 0xffff0000u;
  const float r2 = __fsub_rn(r1, __uint_as_float(mb));
  h = hb >> 16;
  m = mb >> 16;
  l = __float_as_uint(r2) >> 16;
}

// split a pair and pack (x0 -> low half, x1 -> high half) per plane
__device__ inline void split3_pack(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split3(x0, h0, m0, l0);
  split3(x1, h1, m1, l1);
  h = h0 | (h1 << 16);
  m = m0 | (m1 << 16);
  l = l0 | (l1 << 16);
}

// bytes 2b, 2b+1 of w (uint8 pixel values) -> packed bf16 pair (exact)
__device__ inline uint32_t px_pair_bf16(uint32_t w, int b) {
  const float f0 = (float)((w >> (16 * b)) & 0xffu);
  const float f1 = (float)((w >> (16 * b + 8)) & 0xffu);
  return __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
}

// the same exact split of a pair with round-to-nearest pieces: v_cvt_pk_bf16_f32 for each piece, the
// residuals on the packed f32 adder (9 instructions a pair instead of 12).  Exact: x - RN(x) has <= 16
// significant bits, its residual <= 8, so the third piece is exact in bf16 and x = h + m + l.  The pieces
// differ from split3's (rounded, not truncated); the 6-term products are as exact
__device__ inline void split3_pack_rn(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const f2 x = {x0, x1};
  h = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, b2));
  const f2 r1 = x - f2{__uint_as_float(h << 16), __uint_as_float(h & 0xffff0000u)};
  m = __builtin_bit_cast(uint32_t, __builtin_convertvector(r1, b2));
  const f2 r2 = r1 - f2{__uint_as_float(m << 16), __uint_as_float(m & 0xffff0000u)};
  l = __builtin_bit_cast(uint32_t, __builtin_convertvector(r2, b2));
}

// split 8 f32 (one lane's 8 k of a 16x16x32 fragment) into three bf16x8 planes (round-to-nearest pieces:
// fc_bwd 64.3 -> 61.7 us, conv_bwd 106.8 -> 105.2 us in the C4 window against the truncating split, r5m)
__device__ inline void split3_x8(const float (&x)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
  typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
  u32x4_ hh, mm, ll;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t a, b, c;
    split3_pack_rn(x[2 * k], x[2 * k + 1], a, b, c);
    hh[k] = a;
    mm[k] = b;
    ll[k] = c;
  }
  h = __builtin_bit_cast(bf16x8, hh);
  m = __builtin_bit_cast(bf16x8, mm);
  l = __builtin_bit_cast(bf16x8, ll);
}

__device__ inline f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// both split, one accumulator (small terms first): acc += the 6 terms of A.B
__device__ inline f32x4 mfma_x6_acc(bf16x8 ah, bf16x8 am, bf16x8 al, bf16x8 bh, bf16x8 bm, bf16x8 bl, f32x4 acc) {
  acc = mfma_bf16(al, bh, acc);
  acc = mfma_bf16(ah, bl, acc);
  acc = mfma_bf16(am, bm, acc);
  acc = mfma_bf16(am, bh, acc);
  acc = mfma_bf16(ah, bm, acc);
  return mfma_bf16(ah, bh, acc);
}

// A exact in bf16 (pixels), B split: big += A.Bh; small += A.Bl + A.Bm
__device__ inline void mfma_x3(bf16x8 a, bf16x8 bh, bf16x8 bm, bf16x8 bl, f32x4& big, f32x4& small) {
  small = mfma_bf16(a, bl, small);
  small = mfma_bf16(a, bm, small);
  big = mfma_bf16(a, bh, big);
}

// mfma_x3 with the operands' roles swapped: the same exact products and k order, the transposed
// tile (C^T: rows from the split operand, columns from a), so a lane holds 4 consecutive rows of B
__device__ inline void mfma_x3_t(bf16x8 a, bf16x8 bh, bf16x8 bm, bf16x8 bl, f32x4& big, f32x4& small) {
  small = mfma_bf16(bl, a, small);
  small = mfma_bf16(bm, a, small);
  big = mfma_bf16(bh, a, big);
}

// mfma_x6 with the operands' roles swapped (the same products and k order, the transposed tile)
__device__ inline void mfma_x6_t(bf16x8 ah, bf16x8 am, bf16x8 al, bf16x8 bh, bf16x8 bm, bf16x8 bl, f32x4& big,
                                 f32x4& small) {
  small = mfma_bf16(bh, al, small);
  small = mfma_bf16(bm, am, small);
  small = mfma_bf16(bl, ah, small);
  small = mfma_bf16(bh, am, small);
  small = mfma_bf16(bm, ah, small);
  big = mfma_bf16(bh, ah, big);
}

// both split: big += Ah.Bh; small += Al.Bh + Am.Bm + Ah.Bl + Am.Bh + Ah.Bm
__device__ inline void mfma_x6(bf16x8 ah, bf16x8 am, bf16x8 al, bf16x8 bh, bf16x8 bm, bf16x8 bl, f32x4& big,
                               f32x4& small) {
  small = mfma_bf16(al, bh, small);
  small = mfma_bf16(am, bm, small);
  small = mfma_bf16(ah, bl, small);
  small = mfma_bf16(am, bh, small);
  small = mfma_bf16(ah, bm, small);
  big = mfma_bf16(ah, bh, big);
}

template <class T>
__device__ inline T lds_load(const uint8_t* base, int byte_off) {
  return *reinterpret_cast<const T*>(base + byte_off);
}

// 8 bf16 from an 8-byte aligned LDS address (two ds_read_b64)
__device__ inline bf16x8 lds_load8_a8(const uint8_t* base, int byte_off) {
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(base + byte_off);
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(base + byte_off + 8);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace arl
