// Backward of the NIPS head's fully connected layer (dqn_head.py:43,52,
// Linear(2592, 256) + relu) over the S = t_max * n samples of a window
// (a3c.py:129-130):
//   dW[j][k] = sum_s dfc[s][j] a2[s][k],  db[j] = sum_s dfc[s][j]
//   da2[s][k] = (sum_j dfc[s][j] W[j][k]) * (a2[s][k] > 0)
// (dfc is already masked by hfc > 0).  One launch, three independent jobs:
//   job A (dW, db): 128 (j) x 64 (k) tiles over one of Z contiguous sample
//     ranges (Z grows with S, ~800 samples a range).  The Z partials of a
//     tile meet in the same launch: every workgroup publishes its partial
//     (write-through stores, drained) and then takes a ticket; the holder of
//     the last ticket sums the Z partials in range order -- deterministic
//     whatever the arrival order -- straight into the flat gradient (its own
//     from registers, rounded as published).  No workgroup waits on another.  MFMA
//     accumulators restart every 128 samples; those sums add in f64.  db
//     rides on the k-tile 0 workgroups: their n-wave-0 lanes add the A
//     fragments they already hold.
//   job B (da2): 64 (s) x 128 (k) tiles over K = 256, ReLU mask in the
//     epilogue (mask bits prefetched during the k loop, float4 buffer stores).
//   job C (optional): the policy / value heads' weight gradients, a small
//     f64 VALU reduction over S that runs beside A and B instead of as two
//     launches of its own (job_heads below).
// Operands stream HBM/L2 -> LDS by LDS-DMA (global_load_lds dwordx4) into two
// 32 KB stages (K chunks of 32; the next chunk in flight while the current one
// feeds the MFMAs).  A chunk is one 16x16x32 bf16 k-step per tile pair on exact
// bf16 splits of the f32 fragments (bf16split.hpp: 6 MFMAs, f32-accurate; job B
// keeps the 5 small terms in their own accumulator).  256 threads, each wave a
// 64 x 32 (job A) or 32 x 64 (job B) block of 16 x 16 tiles.
// Fragment reads are wide: one lane's 16-byte read of 4 consecutive m (or n)
// feeds 4 MFMA tiles whose rows (columns) interleave with stride 4 (8-byte
// reads: 2 tiles, stride 2).  Job B's A operand is stored k-contiguous and is
// read 4 consecutive k per lane, with the same k order on the B side.
// The DMA writes lane-linear, so an LDS image is XOR-swizzled through the
// global source address (physical 16-byte chunk = logical chunk ^ key) where
// its read pattern would otherwise conflict:
//   job A  A: dfc rows s, 128 floats of j   no key             b128 reads, rows kb + q
//          B: a2 rows s, 64 floats of k     key 8*(row & 1)    b64 reads, rows kb + q
//   job B  A: dfc rows s, 32 floats of j    key (row >> 1) & 7 b128 reads (k-permuted)
//          B: W rows j, 128 floats of k     no key             b128 reads, rows 16g + 4q + r
// (ds_read_b64 serves 32 lanes a cycle over 64 banks, ds_read_b128 16 lanes
// in the groups {0-3, 12-15, 20-27}, ... -- MI355X_MICROARCH.md, LDS).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "arl_internal.hpp"
#include "bf16split.hpp"

namespace arl {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int BUF_DWORD3 = 0x00020000;  // raw buffer resource word 3 (gfx9 family): range-checked, no swizzle
constexpr int OOB = 0x7ffffff0;         // a buffer offset past every range: the access is dropped
constexpr int NT = 256;                 // 4 waves
constexpr int NW = NT / 64;
constexpr int BK = 32;                  // K chunk (rows of a stage)
// job A tile: AJ j x AK k (tiles over all 256 j, a2 streamed once, measured slower: r4p)
constexpr int AJ = 128, AK = 64;
constexpr int AWN = AK / 32;            // job A waves along k (64: 2, 32: 1)
constexpr int STAGE = BK * (AJ + AK) > 8192 ? BK * (AJ + AK) : 8192;   // floats per LDS stage
constexpr int AKEY = AK == 64 ? 1 : 0;  // job A's X image: 64-float rows need the 8 * (row & 1) key, 32-float
                                        // rows are conflict-free (a b64 lane group spans two 128-B rows)
constexpr int BN = 128;                 // job B tile: 32 MT samples x 128 k
constexpr int PART = AJ * AK + AJ;      // floats per published partial (dW tile + db)
constexpr int FLUSH = 4;                // job A: f32 MFMA sums over 4 chunks (128 samples), then f64
static_assert(BK * (AJ + AK) <= STAGE && 128 * BK + BK * BN <= STAGE, "stage size");

// The two layers this kernel serves (the same dual-GEMM shape):
//   dW[j][k] = sum_s dY[s][j] X[s][k] (+ db[j] = sum_s dY[s][j]),
//   dX[s][k] = (sum_j dY[s][j] W[j][k]) * (mask[s][k] > 0)
// ShapeFC: Linear(2592, 256) of the NIPS head (dqn_head.py:43): dY = dfc (S x
//   256), X = a2 (S x 2592), W (256 x 2592), mask = a2, dX = da2.
// ShapeLSTM: the gate weights of L.LSTM(256, 256) (a3c_ale.py:50-51,62;
//   Chainer's LSTM gates = upward(x) + lateral(h)): dY = dG (S x 1024), X =
//   [x | h_prev] (S x 512; h_prev rows of samples whose env reset at that step
//   read 0, as the forward saw them), dW = [upward W | lateral W], db = the
//   upward bias; dX = dfc = (dG Wu) * (hfc > 0).
struct ShapeFC {
  static constexpr int J = HID, KW = A2, KW1 = A2, NB = A2;
  static constexpr bool kLstm = false;
};
struct ShapeLSTM {
  static constexpr int J = GATES, KW = 2 * HID, KW1 = HID, NB = HID;
  static constexpr bool kLstm = true;
};
template <class SH>
struct Dims {
  static constexpr int NJA = SH::J / AJ;              // FC 2, LSTM 8
  static constexpr int NKA = (SH::KW + AK - 1) / AK;  // FC 41 (the last one half full), LSTM 8
  static constexpr int NTA = NJA * NKA;               // job A tiles per range: FC 82, LSTM 64
  static constexpr int NKB = (SH::NB + BN - 1) / BN;  // FC 21 (the last one a quarter full), LSTM 2
  static constexpr int NCHB = SH::J / BK;             // job B K chunks: FC 8, LSTM 32
  static_assert(SH::J % AJ == 0 && SH::J % BK == 0 && SH::KW % 4 == 0 && SH::NB % 4 == 0, "tiles");
  static_assert(SH::KW1 % AK == 0 || SH::KW1 == SH::KW, "a k tile never straddles the two dW blocks");
};
static_assert(A2 % AK == 32 || A2 % AK == 0, "FC: the last job A k tile is half or wholly full");
constexpr int NTA_MAX = Dims<ShapeFC>::NTA;
static_assert(Dims<ShapeLSTM>::NTA <= NTA_MAX, "ticket / partial workspace");
constexpr int RST_MAX = 1024;           // LSTM job A: reset flags of a sample range, staged in LDS

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// XCD-aware job order.
// Workgroups are dealt round-robin over the 8 XCDs (b % 8 share one XCD and
// its L2; which XCD is not fixed, MI355X_MICROARCH.md), so job b of n gets
// linear work index xcd_order(b, n): every XCD takes one contiguous range of
// the linear order.  Linear orders put tiles that share an operand next to
// each other -- job A: the two j tiles of one (range, k tile) a2 slice; job B:
// the sample tiles of one k tile (one W slice) -- so each slice is fetched
// into about one L2 instead of all eight.
__device__ inline int xcd_order(int b, int n) {
  const int x = b & 7, slot = b >> 3, per = n >> 3, rem = n & 7;
  return x * per + min(x, rem) + slot;
}

__device__ inline uint64_t pack2(float lo, float hi) {
  return (uint64_t)__float_as_uint(lo) | ((uint64_t)__float_as_uint(hi) << 32);
}

__device__ inline void barrier_lds() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Stage R rows x WC floats of a row-major matrix into LDS at dst by LDS-DMA:
// tile row r = global row min(row0 + r, rmax); logical 16-byte chunk c of
// row r lands at physical chunk c ^ key(r).  Wave w issues the 1 KB pieces
// w, w + NW, ...
// ZR (LSTM h_prev): rows whose flag zr[row - zbase] is set (LDS) read the zero row instead.
template <int R, int WC, int KEY, bool ZR = false>
__device__ inline void stage_tile(float* dst, const float* __restrict__ g, int64_t ld, int row0, int rmax, int col0,
                                  const uint8_t* zr = nullptr, int zbase = 0, const float* zero = nullptr) {
  constexpr int CPR = WC / 4;                 // chunks per row
  constexpr int NI = R * WC * 4 / 1024;       // 1 KB pieces
  static_assert(NI % NW == 0, "whole pieces per wave");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int ii = 0; ii < NI / NW; ++ii) {
    const int it = ii * NW + wave;
    const int i = it * 64 + lane;             // chunk index in the tile image
    const int r = i / CPR, pc = i - r * CPR;
    int key = 0;
    if constexpr (KEY == 1) key = 8 * (r & 1);
    else if constexpr (KEY == 2) key = (r >> 1) & 7;
    const int row = min(row0 + r, rmax);
    const float* src = g + (int64_t)row * ld + col0 + 4 * (pc ^ key);
    if constexpr (ZR) {
      if (zr[row - zbase]) src = zero + 4 * (pc ^ key);
    }
    __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)(dst + it * 256), 16, 0, 0);
  }
}

struct FcBwdArgs {
  const float* dfc;   // dY: (S, 256) FC / dG (S, 1024) LSTM
  const float* a2;    // X (FC: (S + 1, 2592): job A's last k tile reads 32 floats past a row's end);
                      // LSTM: x = hfc (S, 256), also the ReLU mask of both
  const float* W;     // (256, 2592) followed by more parameters / LSTM Wu (1024, 256)
  int S, Z, kpz;      // job A: Z sample ranges of kpz samples (multiple of BK)
  float* gW;          // (256, 2592) / LSTM upward W (1024, 256)
  float* gb;          // (256) / LSTM upward b (1024)
  float* da2;         // dX: (S, 2592) / LSTM dfc (S, 256)
  float* part;        // (NTA, Z, PART) published job A partials (slot z = range z)
  int* tick;          // (NTA): arrival tickets per tile
  HeadsDW hd;         // job C (hd.dl null: none)
  int nc;             // job C workgroups
  // LSTM only
  const float* hprev;      // h_prev (S, 256): the carry-in h of each sample's step (hbuf slot t)
  const uint8_t* reset;    // (S): the env reset at that step (its h_prev reads 0)
  const float* zero;       // >= 64 zero floats (the DMA source of a reset row)
  float* gW2;              // lateral W (1024, 256)
  // FC: job B's ReLU mask as bits of a2 > 0 (S, 81 words; conv_fwd.hip writes them) instead of a2
  // itself -- 324 instead of 10,368 bytes a sample; null: read a2
  const uint32_t* a2m = nullptr;
};

// ---------------------------------------------------------------- job A: dW, db
template <class SH>
__device__ void job_dw(const FcBwdArgs& a, int job, float* lds, uint8_t* rst) {
  using D = Dims<SH>;
  constexpr int NTA = D::NTA;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, col = lane & 15;
  const int wm = wave / AWN, wn = wave % AWN;   // wave: 64 j x 32 k
  // linear order (z, kt, jt), jt fastest, dealt to the XCDs in contiguous ranges
  const int lin = xcd_order(job, NTA * a.Z);
  const int z = lin / NTA;
  const int tile = ((lin - z * NTA) % D::NJA) * D::NKA + (lin - z * NTA) / D::NJA;
  const int kt = tile % D::NKA, jt = tile / D::NKA;
  const int j0 = jt * AJ, k0 = kt * AK;
  const int r0 = z * a.kpz, r1 = min(a.S, r0 + a.kpz);
  const bool bias = kt == 0 && wn == 0;
  const int nchunks = max(0, (r1 - r0 + BK - 1) / BK);
  // X columns of this k tile: FC a2; LSTM x = hfc (k < 256) or h_prev (k >= 256, the
  // range's reset flags staged in LDS first: a reset sample's row is DMA'd from the zero row)
  const bool hpart = SH::kLstm && k0 >= SH::KW1;   // block-uniform
  const float* xsrc = hpart ? a.hprev : a.a2;
  constexpr int XLD = SH::kLstm ? HID : A2;
  const int xc0 = hpart ? k0 - SH::KW1 : k0;
  if (hpart) {
    for (int i = tid; i < r1 - r0; i += NT) rst[i] = a.reset[r0 + i];
    __syncthreads();
  }
  // m-tile t: rows j = wm*64 + 4 col + t; n-tile u: cols k = wn*32 + 2 col + u
  double s[4][2][4], sb[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    sb[t] = 0.0;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) s[t][u][e] = 0.0;
  }
  auto issue = [&](int c) {
    float* st = lds + (c & 1) * STAGE;
    stage_tile<BK, AJ, 0>(st, a.dfc, SH::J, r0 + c * BK, r1 - 1, j0);       // dY[s][j0 .. j0+127]
    if (SH::kLstm && hpart)
      stage_tile<BK, AK, AKEY, true>(st + BK * AJ, xsrc, XLD, r0 + c * BK, r1 - 1, xc0, rst, r0, a.zero);
    else
      stage_tile<BK, AK, AKEY>(st + BK * AJ, xsrc, XLD, r0 + c * BK, r1 - 1, xc0);   // X[s][k0 .. k0+AK-1]
  };
  const int nb = wn * 32 + 2 * col;
  f32x4 acc[4][2], bs;
  if (nchunks > 0) issue(0);
  for (int c = 0; c < nchunks; ++c) {
    // one barrier a chunk: past it, every wave has this chunk's DMA landed
    // (its own pieces drained before the barrier) and has finished reading
    // the other stage (chunk c - 1), which the next chunk's DMA then fills.
    // (A third stage, two chunks in flight, measured no faster.)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // (lgkm: chunk c - 1's LDS reads returned)
    barrier_lds();
    if (c + 1 < nchunks) issue(c + 1);
    const float* As = lds + (c & 1) * STAGE;
    const float* Bs = As + BK * AJ;
    const int kvalid = r1 - (r0 + c * BK);   // rows >= kvalid: clamped copies, masked to 0
    if (c % FLUSH == 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
      bs = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    {
      // every fragment of the chunk first (counted LDS waits), then the MFMAs
      f32x4 av[BK / 4];
      f32x2 bv[BK / 4];
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        const int r = 4 * ks + q;
        av[ks] = *reinterpret_cast<const f32x4*>(As + r * AJ + wm * 64 + 4 * col);
        bv[ks] = *reinterpret_cast<const f32x2*>(Bs + r * AK + (((nb >> 2) ^ (AKEY * 8 * (r & 1))) << 2) + (nb & 3));
      }
      if (kvalid < BK) {   // the range's last chunk only
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks)
          if (4 * ks + q >= kvalid) av[ks] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      {
        // one 16x16x32 bf16 step per tile pair: element i of lane (col, q) is sample 4 i + q
        bf16x8 bh[2], bm[2], bl[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float x[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = bv[i][u];
          split3_x8(x, bh[u], bm[u], bl[u]);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float x[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = av[i][t];
          bf16x8 ah, am, al;
          split3_x8(x, ah, am, al);
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[t][u] = mfma_x6_acc(ah, am, al, bh[u], bm[u], bl[u], acc[t][u]);
        }
        if (bias)
#pragma unroll
          for (int ks = 0; ks < BK / 4; ++ks) bs += av[ks];
      }
    }
    if (c % FLUSH == FLUSH - 1 || c == nchunks - 1) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        sb[t] += (double)bs[t];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) s[t][u][e] += (double)acc[t][u][e];
      }
    }
  }
  // C layout (16x16x4): lane (col, q) holds rows 4q + e, column col of each
  // tile -> j = j0 + wm*64 + 16q + 4e + t, k = k0 + wn*32 + 2col + u
  if (bias) {   // lanes (col, q) hold sums over rows = q (mod 4): fixed-order quarter reduction
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      double v = sb[t];
      v = v + __shfl_xor(v, 16);
      sb[t] = v + __shfl_xor(v, 32);
    }
  }
  auto pidx = [&](int t, int u, int e) { return (wm * 64 + 16 * q + 4 * e + t) * AK + wn * 32 + 2 * col + u; };
  if (a.Z > 1) {
    // every range publishes into its slot (write-through sc1 stores, drained),
    // then takes a ticket; the holder of the last ticket sums the slots.
    // Ordering: this is the hand-off MI355X_MICROARCH.md lists as valid on
    // gfx950 / ROCm 7.2 without an agent release / acquire pair (its table of
    // sc1 hand-offs, first row): every byte stored sc1 and drained by its
    // storing wave (vmcnt(0)) before the workgroup barrier, one lane's
    // agent-scope ticket add, and the last holder reading every slot with sc1
    // loads only after its add returned.  Measured hardware behaviour, not
    // the HIP memory model: a release fence here (buffer_wbl2, ~1.7-6.5 us per
    // workgroup) is what the model would need on another target.
    float* dst = a.part + ((int64_t)tile * a.Z + z) * PART;
    // the (u = 0, 1) pair of a lane is 8 contiguous bytes: one 64-bit store,
    // so a quarter-wave writes 128 contiguous bytes (whole sectors)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __hip_atomic_store(reinterpret_cast<uint64_t*>(dst + pidx(t, 0, e)), pack2((float)s[t][0][e], (float)s[t][1][e]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (bias && q == 0)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        __hip_atomic_store(dst + AJ * AK + wm * 64 + 4 * col + t, (float)sb[t], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds);   // the stages are free after the k loop's last barrier
    if (tid == 0) {
      const int tk = __hip_atomic_fetch_add(&a.tick[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = tk == a.Z - 1;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // every slot load below is sc1
  }
  // sum the Z partials in range order (own range from registers, rounded as
  // published), f64; two slots' loads in flight at a time
  double o[4][2][4], ob[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    ob[t] = 0.0;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) o[t][u][e] = 0.0;
  }
  for (int z2 = 0; z2 < a.Z; z2 += 2) {
    float v[2][4][2][4], vb[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int zz = min(z2 + h, a.Z - 1);
      const float* src = a.part + ((int64_t)tile * a.Z + zz) * PART;
      if (zz == z) {   // one wave-uniform branch per slot: every load of a slot in flight together
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          vb[h][t] = (float)sb[t];
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[h][t][u][e] = (float)s[t][u][e];
        }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          vb[h][t] = __hip_atomic_load(src + AJ * AK + wm * 64 + 4 * col + t, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);   // (garbage off the bias waves: unused)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint64_t w = __hip_atomic_load(reinterpret_cast<const uint64_t*>(src + pidx(t, 0, e)),
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v[h][t][0][e] = __uint_as_float((unsigned)w);
            v[h][t][1][e] = __uint_as_float((unsigned)(w >> 32));
          }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (z2 + h >= a.Z) break;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        ob[t] += (double)vb[h][t];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) o[t][u][e] += (double)v[h][t][u][e];
      }
    }
  }
  const int k = k0 + wn * 32 + 2 * col;
  if (k < SH::KW) {   // FC: the last k tile is half full (k even, A2 even: a pair is all in or out)
    // LSTM: k < 256 the upward W, else the lateral W (a k tile never straddles the two)
    float* gw = hpart ? a.gW2 + (k - SH::KW1) : a.gW + k;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = j0 + wm * 64 + 16 * q + 4 * e + t;
        float2 w;
        w.x = (float)o[t][0][e];
        w.y = (float)o[t][1][e];
        *reinterpret_cast<float2*>(gw + (int64_t)j * SH::KW1) = w;
      }
  }
  if (bias && q == 0)
#pragma unroll
    for (int t = 0; t < 4; ++t) a.gb[j0 + wm * 64 + 4 * col + t] = (float)ob[t];
  if (a.Z > 1 && tid == 0)   // re-arm for the next launch (a captured graph replays this one)
    __hip_atomic_store(&a.tick[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- job B: da2
// MT m-tiles per wave: workgroup tiles of BMT = 32 MT samples x 128 k
template <int MT, class SH, bool BITS>
__device__ void job_da2(const FcBwdArgs& a, int tile, float* lds) {
  using D = Dims<SH>;
  constexpr int NKB = D::NKB, NB = SH::NB;
  constexpr int BMT = 32 * MT;
  constexpr int PIECES = (BMT * BK + BK * BN) / 256 / NW;   // LDS-DMA pieces per wave per chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, col = lane & 15;
  const int wm = wave >> 1, wn = wave & 1;   // wave: 16 MT s x 64 k
  // linear order (kt, st), st fastest, dealt to the XCDs in contiguous ranges
  const int nst = (a.S + BMT - 1) / BMT;
  const int lin = xcd_order(tile, nst * NKB);
  const int kt = lin / nst, st = lin - kt * nst;
  const int s0 = st * BMT, k0 = kt * BN;
  constexpr int NCH = D::NCHB;               // chunks of 32 j: FC 8, LSTM 32
  auto issue = [&](int c) {
    float* sg = lds + (c & 1) * STAGE;
    stage_tile<BMT, BK, 2>(sg, a.dfc + c * BK, SH::J, s0, a.S - 1, 0);                  // dY[s][j]
    stage_tile<BK, BN, 0>(sg + BMT * BK, a.W + (int64_t)c * BK * NB, NB, 0, BK - 1, k0);  // W[j][k0..k0+127]
  };
  f32x4 acc[MT][4];                          // m-tile i: rows 16 i + col; n-tile u: cols 4 col + u
  f32x4 sml[MT][4];                          // the 5 small terms (acc: the h.h term)
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int u = 0; u < 4; ++u) sml[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  // ReLU mask of the tile (a2 > 0), one bit per output element -- bit 4e + u
  // of mb[i] -- loaded a 16-row band per chunk during chunks 0..MT-1 so that no
  // load round trip is left for the epilogue.  Out-of-range rows / columns
  // read 0 through the buffer's range check.
  const int k = k0 + wn * 64 + 4 * col;
  const bool kin = k < NB;                   // NB % 4 == 0: a 4-run is all in or all out
  const int rows = min(BMT, a.S - s0);
  const __amdgpu_buffer_rsrc_t msk = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.a2) + (int64_t)s0 * NB,
                                                                       0, rows * NB * 4, BUF_DWORD3);
  unsigned mb[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) mb[i] = 0u;
  f32x4 mraw[4];
  uint32_t mw[4];
  constexpr bool bits = BITS;   // (compile-time: a runtime choice branches around every mask load, each waiting
                                //  for all DMA in flight)
  const __amdgpu_buffer_rsrc_t mskw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(bits ? a.a2m : nullptr) + (int64_t)s0 * A2W, 0, bits ? rows * A2W * 4 : 0, BUF_DWORD3);
  issue(0);
#pragma unroll 8
  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) issue(c + 1);
    if (c >= 1 && c <= MT) {   // the band loaded one chunk ago (the compiler's own vmcnt wait)
      if (bits) {
#pragma unroll
        for (int e = 0; e < 4; ++e) mb[c - 1] |= ((mw[e] >> (k & 31)) & 0xfu) << (4 * e);   // k % 4 == 0
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int u = 0; u < 4; ++u) mb[c - 1] |= (mraw[e][u] > 0.f ? 1u : 0u) << (4 * e + u);
      }
    }
    if (c < MT) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * 16 * MT + 16 * c + 4 * q + e;
        if (bits)
          mw[e] = __builtin_amdgcn_raw_buffer_load_b32(mskw, kin ? (row * A2W + (k >> 5)) * 4 : OOB, 0, 0);
        else
          mraw[e] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(msk, kin ? (row * NB + k) * 4 : OOB, 0, 0));
      }
    }
    // this chunk's DMA done: the next chunk's PIECES a wave and this chunk's mask band may still fly
    if (c + 1 < NCH) {
      if (c < MT) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES + 4) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier_lds();
    const float* As = lds + (c & 1) * STAGE;
    const float* Bs = As + BMT * BK;
    {
      // every fragment of the chunk first (counted LDS waits), then the MFMAs
      f32x4 av[BK / 16][MT], bv[BK / 16][4];
#pragma unroll
      for (int g = 0; g < BK / 16; ++g) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const int m = wm * 16 * MT + i * 16 + col;
          av[g][i] = *reinterpret_cast<const f32x4*>(As + m * BK + (((4 * g + q) ^ ((m >> 1) & 7)) << 2));
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)   // k = 16 g + 4 q + r on both operands
          bv[g][r] = *reinterpret_cast<const f32x4*>(Bs + (16 * g + 4 * q + r) * BN + wn * 64 + 4 * col);
      }
      {
        // one 16x16x32 bf16 step per tile pair: element 4 g + r of lane
        // (col, q) is k = 16 g + 4 q + r on both operands
        bf16x8 bh[4], bm[4], bl[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float x[8];
#pragma unroll
          for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) x[4 * g + r] = bv[g][r][u];
          split3_x8(x, bh[u], bm[u], bl[u]);
        }
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          float x[8];
#pragma unroll
          for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) x[4 * g + r] = av[g][i][r];
          bf16x8 ah, am, al;
          split3_x8(x, ah, am, al);
#pragma unroll
          for (int u = 0; u < 4; ++u) mfma_x6(ah, am, al, bh[u], bm[u], bl[u], acc[i][u], sml[i][u]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier_lds();
  }
  // lane (col, q) holds s = s0 + wm*16*MT + 16 i + 4 q + e, k = k0 + wn*64 + 4 col + u:
  // 4 consecutive k per (i, e).  Straight-line buffer stores whose
  // out-of-range lanes (s >= S, k >= A2) the buffer's range check drops -- no
  // per-store branch, so no store waits for the one before it.
  const __amdgpu_buffer_rsrc_t out =
      __builtin_amdgcn_make_buffer_rsrc(a.da2 + (int64_t)s0 * NB, 0, rows * NB * 4, BUF_DWORD3);
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = wm * 16 * MT + 16 * i + 4 * q + e;
      f32x4 o;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float v = acc[i][u][e] + sml[i][u][e];
        o[u] = (mb[i] >> (4 * e + u)) & 1u ? v : 0.f;
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), out, kin ? (row * NB + k) * 4 : OOB, 0, 0);
    }
}

// ---------------------------------------------------------------- job C: heads dW, db
// Workgroup jt: columns j = 16 jt + (tid & 15) of h; the 16 thread rows
// p = tid >> 4 take the samples s = p (mod 16), four samples' loads in flight
// before their FMAs, and accumulate rows a = 0..A (dlogits columns, then dv)
// in f64, 8 rows a pass.  The partitions meet in LDS and are summed in order.
// Column 16 of workgroup 0 is the bias (h = 1), summed by its column-0 threads.
constexpr int CW = 16, NP = NT / CW;     // 16 columns x 16 sample partitions
constexpr int NJC = HID / CW;            // 16 workgroups
__device__ void job_heads(const FcBwdArgs& a, int jt, float* lds) {
  const HeadsDW& d = a.hd;
  const int tid = threadIdx.x, jj = tid % CW, p = tid / CW;
  const int j = jt * CW + jj;
  const int R = d.A + 1;
  const bool bias = jt == 0 && jj == 0;
  double* red = reinterpret_cast<double*>(lds);   // [NP][8][CW + 1] partials
  for (int a0 = 0; a0 < R; a0 += 8) {
    double acc[8], accb[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = accb[r] = 0.0;
    for (int s0 = p; s0 < a.S; s0 += 4 * NP) {
      float hv[4], gv[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {   // every load first (clamped rows, zero weight past S)
        const int s = min(s0 + u * NP, a.S - 1);
        const float ok = s0 + u * NP < a.S ? 1.f : 0.f;
        hv[u] = d.h[(int64_t)s * HID + j] * ok;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int row = min(a0 + r, d.A);
          gv[u][r] = (row < d.A ? d.dl[(int64_t)s * d.A + row] : d.dv[s]) * ok;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          acc[r] = fma((double)gv[u][r], (double)hv[u], acc[r]);
          accb[r] += (double)gv[u][r];
        }
    }
    __syncthreads();   // the previous pass's partials are consumed
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      red[(p * 8 + r) * (CW + 1) + jj] = acc[r];
      if (bias) red[(p * 8 + r) * (CW + 1) + CW] = accb[r];
    }
    __syncthreads();
    for (int i = tid; i < 8 * (CW + 1); i += NT) {   // (row, column) of this pass, partitions in order
      const int r = i / (CW + 1), c = i - r * (CW + 1), row = a0 + r;
      if (row >= R || (c == CW && jt != 0)) continue;
      double v = 0.0;
      for (int q = 0; q < NP; ++q) v += red[(q * 8 + r) * (CW + 1) + c];
      if (c < CW) {
        if (row < d.A) d.gWpi[(int64_t)row * HID + jt * CW + c] = (float)v;
        else d.gWv[jt * CW + c] = (float)v;
      } else {
        if (row < d.A) d.gbpi[row] = (float)v;
        else d.gbv[0] = (float)v;
      }
    }
  }
}

template <int MT, class SH, bool BITS>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2)))
fc_bwd_kernel(FcBwdArgs a) {
  // 64 KB of stages + (LSTM) a range's reset flags in one __shared__ object: a second one beside the
  // LDS-DMA staging makes the compiler drain every DMA in flight (vmcnt(0)) before a chunk's LDS reads
  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE + (SH::kLstm ? RST_MAX / 4 : 0)];
  uint8_t* rst = reinterpret_cast<uint8_t*>(lds + 2 * STAGE);
  const int b = blockIdx.x;
  const int na = Dims<SH>::NTA * a.Z;
  if (b < a.nc) job_heads(a, b, lds);   // first: the smallest, longest-latency jobs
  else if (b < a.nc + na) job_dw<SH>(a, b - a.nc, lds, rst);
  else job_da2<MT, SH, BITS>(a, b - a.nc - na, lds);
}

// ~800 samples per job A range, at most 16 ranges (bf16-split steps, sweep in
// profiles/r02/fcb_split/z_sweep.txt: best Z 2 / 3-5 / 6 at S 1280 / 2560 / 5120)
int fc_bwd_ranges(int S) {
  return std::max(1, std::min(16, (S + 400) / 800));
}
// LSTM: the same, with no range longer than the LDS reset table
int lstm_wgrad_ranges(int S) { return std::max(fc_bwd_ranges(S), (S + RST_MAX - 1) / RST_MAX); }
int range_len(int S, int Z) { return ((S + Z - 1) / Z + BK - 1) / BK * BK; }
}  // namespace

int64_t fc_bwd_part_floats(int S) {
  return (int64_t)std::max(Dims<ShapeFC>::NTA * fc_bwd_ranges(S), Dims<ShapeLSTM>::NTA * lstm_wgrad_ranges(S)) * PART;
}
int fc_bwd_tickets() { return NTA_MAX; }   // arrival tickets

// Job A's last k tile stages a2 columns 2560..2623 and job B's last one W
// columns 2560..2687: the floats past a row's end are the next row's (a2 has
// the bootstrap slot after the window's S rows) or the next parameters' (W),
// and are never stored.
hipError_t launch_fc_bwd(const float* dfc, const float* a2, const float* W, int S, float* gW, float* gb, float* da2,
                         float* part, int* tick, hipStream_t s, const HeadsDW* heads, const uint32_t* a2m) {
  if (S <= 0) return hipSuccess;
  const int Z = fc_bwd_ranges(S);
  const int kpz = range_len(S, Z);
  // job B tiles: 64 samples (2 m-tiles a wave; the small-term accumulators leave no room for 4)
  constexpr int MT = 2, BMT = 32 * MT;
  using D = Dims<ShapeFC>;
  const int na = D::NTA * Z, nb = ((S + BMT - 1) / BMT) * D::NKB;
  if (heads != nullptr && (heads->A < 1 || heads->dl == nullptr)) return hipErrorInvalidValue;
  const int nc = heads != nullptr ? NJC : 0;
  FcBwdArgs args{dfc, a2, W, S, Z, kpz, gW, gb, da2, part, tick, heads ? *heads : HeadsDW{}, nc,
                 nullptr, nullptr, nullptr, nullptr, a2m};
  if (a2m != nullptr) hipLaunchKernelGGL((fc_bwd_kernel<MT, ShapeFC, true>), dim3(nc + na + nb), dim3(NT), 0, s, args);
  else hipLaunchKernelGGL((fc_bwd_kernel<MT, ShapeFC, false>), dim3(nc + na + nb), dim3(NT), 0, s, args);
  return hipGetLastError();
}

// LSTM gate weight gradients + dfc in one launch (ShapeLSTM above): job A
// writes the upward W / b and lateral W gradients straight into the flat
// gradient, job B dfc = (dG Wu) * (hfc > 0).  zero: >= 64 zero floats.
hipError_t launch_lstm_wgrad(const float* dG, const float* hfc, const float* hprev, const uint8_t* reset,
                             const float* zero, const float* Wu, int S, float* gWu, float* gWl, float* gbu, float* dfc,
                             float* part, int* tick, hipStream_t s) {
  if (S <= 0) return hipSuccess;
  const int Z = lstm_wgrad_ranges(S);
  const int kpz = range_len(S, Z);
  if (kpz > RST_MAX) return hipErrorInvalidValue;
  using D = Dims<ShapeLSTM>;
  constexpr int BMT = 64;
  const int na = D::NTA * Z, nb = ((S + BMT - 1) / BMT) * D::NKB;
  FcBwdArgs args{dG, hfc, Wu, S, Z, kpz, gWu, gbu, dfc, part, tick, HeadsDW{}, 0, hprev, reset, zero, gWl};
  hipLaunchKernelGGL((fc_bwd_kernel<2, ShapeLSTM, false>), dim3(na + nb), dim3(NT), 0, s, args);
  return hipGetLastError();
}

}  // namespace arl
