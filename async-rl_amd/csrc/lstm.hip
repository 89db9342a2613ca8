// The LSTM's gate GEMM with the cell in its epilogue (a3c_ale.py:50-51,62:
// L.LSTM(256, 256) = upward Linear(256, 1024) + lateral Linear(256, 1024, no
// bias) -> Chainer 1.8.1 F.lstm; one launch per lockstep step):
//
//   gates[m][j] = (x[m] . Wu[j] + b[j]) + (reset[m] ? 0 : h[m] . Wl[j])   (Chainer's order:
//                 upward(x) with its bias, then + lateral(h))
//   (a, i, f, o) = gates[m][4u .. 4u + 3]          (interleaved, reshape(n, 256, 4))
//   c' = tanh(a) sig(i) + sig(f) c,   h' = sig(o) tanh(c')
//
// M = n envs, N = 1024 gate columns, K = 512 = [x | h].  Shaped like fc.hip
// (latency-bound at these sizes: one short chain per workgroup):
//   * 32 x 64 output tile (16 units x 4 gates) per 512-thread workgroup, 8
//     waves with one 16 x 16 sub-tile each (exact f32 v_mfma_f32_16x16x4_f32);
//   * the 96 operand rows (32 of [x | h], 64 of [Wu | Wl]) are staged by
//     LDS-DMA in four 128-column K chunks through three LDS stages (row stride
//     33 float4: the 16 rows a ds_read_b128 touches land on distinct bank
//     quads); chunks 0-2 are issued at once, chunk 3 as soon as stage 0 is free;
//   * the x and h halves accumulate separately, so a reset row (h = None after
//     an episode end, a3c.py:166 / a3c_ale.py:65-66) drops the h half at the
//     epilogue instead of zero-filling staged rows;
//   * epilogue: the tile through LDS (row stride 68 floats: the four lane
//     quarters' rows on distinct banks; the bias added before it), one (row,
//     unit) per thread: the gates written for the backward, and the cell -- the arithmetic of
//     lstm_cell_fwd_kernel (net.hip), op for op.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "arl_internal.hpp"

namespace arl {

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int LBM = 32, LBN = 64, LT = 512, LW = LT / 64;
constexpr int LKC = 128;                       // K chunk (columns)
constexpr int LROWS = LBN + LBM;               // 96 staged rows: 64 of [Wu | Wl], then 32 of [x | h]
// float4 per staged row (32 used): 34 = 2 mod 16, so the 8 + 8 rows of a ds_read_b128 lane group's two
// 16-byte k quarters land on 16 distinct bank quads (33 = 1 mod 16 puts two of them on one quad); the
// same for the BPTT kernel's dG rows (BA_LD).  34 vs 33 at C3: lstm_gates 20.3 -> 19.2 us, lstm_bptt
// 17.1 -> 16.8 us, window 1.151 -> 1.140 ms (profiles/r04/r4o)
constexpr int LSTM_LD = 34;
// the saved gate pre-activations (read only by the window's BPTT) stored non-temporal, as conv_fwd's a1 / a2:
// C3 median 1.1133 / 1.1144 -> 1.1091 / 1.1109 ms, lstm_gates 19.5 -> 19.1 us (2 interleaved reps, r4t)
constexpr int LLD = LSTM_LD;
constexpr int LPIECES = (LROWS * LLD + 63) / 64;   // 51 LDS-DMA pieces (64 x 16 B) per chunk
constexpr int LWPIECES = LBN * LLD / 64;       // 34: the W rows alone (XRED x chunks)
constexpr int LSTAGE4 = LPIECES * 64;          // float4 per stage (incl. the last piece's overhang)
constexpr int LSTAGES = 3;
constexpr int TLD = 68;                        // epilogue tile row stride (floats)
static_assert(LBN * LLD % 64 == 0, "the A rows start on a piece boundary");
static_assert(LBM * TLD <= LSTAGE4 * 4, "epilogue tile fits one stage");
static_assert(GATES % LBN == 0 && LBM * (LBN / 4) == LT, "one (row, unit) per thread");
// every wave issues the same number of pieces per chunk (pieces past the end
// repeat the last one: the same bytes to the same LDS slots), so the counted
// waits below are compile-time constants and the compiler's own wait for
// the XRED partial loads counts exactly the DMA issued after them
constexpr int LPW = (LPIECES + LW - 1) / LW;   // 7
constexpr int LWPW = (LWPIECES + LW - 1) / LW; // 5
constexpr int XRJ = LBM * HID / 4 / LT;        // XRED: float4 of the x tile per thread (4)
}  // namespace

// s_waitcnt vmcnt(n) for the compile-time counts of the LSTM kernels
template <int N>
__device__ inline void lstm_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-only workgroup barrier (keeps the other chunks' LDS-DMA in flight; see conv_bwd.hip)
__device__ inline void lstm_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ inline float lstm_sigm(float x) { return __fdiv_rn(1.f, __fadd_rn(1.f, expf(-x))); }

struct LstmGatesArgs {
  const float* x;        // (n, 256) the upward input (the FC output); XRED: unused
  const float* h;        // (n, 256) h_prev (ignored on reset rows)
  const uint8_t* reset;  // (n) 1 = the state is None
  const float* Wu;       // (1024, 256)
  const float* Wl;       // (1024, 256)
  const float* b;        // (1024)
  float* gates;          // (n, 1024) pre-activations (+ bias), kept for the backward
  const float* c_prev;   // (n, 256)
  float* c_out;          // (n, 256) (cell == 0: untouched)
  float* h_out;          // (n, 256)
  // XRED: x = relu(sum_z slab[z] + fc_b) formed here from the FC forward's
  // split-K partials (fc.hip, tickets == nullptr), summed in split order
  // 0..7 from 0.f like fc_fwd_kernel's last arriver (bit-identical hfc);
  // the column-tile-0 workgroups write it to hfc for the backward
  const float* slab;     // (FC_SPLIT, n, 256)
  const float* fc_b;     // (256)
  float* hfc;            // (n, 256)
  int n, cell;
};

template <bool XRED>
__global__ void __launch_bounds__(LT)
lstm_gates_kernel(LstmGatesArgs a) {
  __shared__ __attribute__((aligned(16))) float S[LSTAGES * LSTAGE4 * 4];   // 156,672 B
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NTN = GATES / LBN;
  const int m0 = (blockIdx.x / NTN) * LBM, n0 = (blockIdx.x % NTN) * LBN;

  // ---- staging: chunk c into stage c % 3; slot i -> row i / LLD, float4
  // column min(i % LLD, 31) (the pad slot re-loads the row's last float4);
  // rows 0..63 are W rows n0.., rows 64..95 env rows m0.. (XRED chunks 0, 1:
  // the W rows only, the x rows are written from registers)
  auto issue = [&](int c) {
    float* st = S + 4 * LSTAGE4 * (c % LSTAGES);
    const int kc = (c & 1) * LKC;
    const float* xa = c < 2 ? a.x : a.h;
    const float* wb = c < 2 ? a.Wu : a.Wl;
    const bool wonly = XRED && c < 2;
    const int np = wonly ? LWPIECES : LPIECES;
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      if (wonly && j >= LWPW) break;   // uniform: c is a compile-time constant at every call
      const int it = min(wave + LW * j, np - 1);
      const int i = min(it * 64 + lane, LROWS * LLD - 1);
      const int r = i / LLD, cc = min(i - r * LLD, LKC / 4 - 1);
      const float* src = r < LBN ? wb + (int64_t)(n0 + r) * HID
                                 : xa + (int64_t)min(m0 + r - LBN, a.n - 1) * HID;   // rows past n: any valid row
      __builtin_amdgcn_global_load_lds(src + kc + 4 * cc, (__attribute__((address_space(3))) void*)(st + 4 * it * 64),
                                       16, 0, 0);
    }
  };
  const int q = lane >> 4, col = lane & 15;
  const int ms = wave & 1, ns = wave >> 1;
  // reset flags of this lane's four C rows, issued first (the oldest loads, so
  // the counted waits below cover them with chunk 0)
  uint8_t rs[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) rs[r] = a.reset[min(m0 + ms * 16 + q * 4 + r, a.n - 1)];
  typedef float xf4 __attribute__((ext_vector_type(4)));
  f32x4 accx = {0.f, 0.f, 0.f, 0.f}, acch = accx;
  auto compute = [&](int c, f32x4& acc) {
    const float* st = S + 4 * LSTAGE4 * (c % LSTAGES);
    const float* Ar = st + (LBN + ms * 16 + col) * 4 * LLD + 4 * q;
    const float* Br = st + (ns * 16 + col) * 4 * LLD + 4 * q;
    // lane quarter q holds k = 16 s + 4 q + r of the chunk; the fragments of
    // four s read first (one LDS wait), then their 16 MFMAs back to back
#pragma unroll
    for (int s0 = 0; s0 < LKC / 16; s0 += 4) {
      f32x4 av[4], bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        av[s] = *reinterpret_cast<const f32x4*>(Ar + 16 * (s0 + s));
        bv[s] = *reinterpret_cast<const f32x4*>(Br + 16 * (s0 + s));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s][r], bv[s][r], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  xf4 xo[XRED ? XRJ : 1];
  if constexpr (XRED) {
    // chunks 0-2 go out first (chunks 0, 1: the W rows only), then the x
    // tile's FC partials and bias (float4 idx = tid + 512 j: row idx / 64,
    // float4 column idx % 64), summed as they land; every operand is in
    // flight at once, so waiting for all of it before chunk 0's MFMAs costs
    // little (the staging is latency-bound), and the compiler's own waits for
    // the partials (it does not count LDS-DMA) stay correct whatever order
    // it issues them in
    issue(0);
    issue(1);
    issue(2);
    // (scheduling barriers: every DMA piece, then every partial load, issued
    // before the first add -- one wait for all of them)
    __builtin_amdgcn_sched_barrier(0);
    xf4 p[XRJ][FC_SPLIT], b[XRJ];
#pragma unroll
    for (int j = 0; j < XRJ; ++j) {
      const int idx = tid + LT * j, row = idx >> 6, c4 = idx & 63;
      const int64_t m = min(m0 + row, a.n - 1);
#pragma unroll
      for (int z = 0; z < FC_SPLIT; ++z)
        p[j][z] = *reinterpret_cast<const xf4*>(a.slab + ((int64_t)z * a.n + m) * HID + 4 * c4);
      b[j] = *reinterpret_cast<const xf4*>(a.fc_b + 4 * c4);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < XRJ; ++j) {
      xf4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int z = 0; z < FC_SPLIT; ++z)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = __fadd_rn(acc[e], p[j][z][e]);
#pragma unroll
      for (int e = 0; e < 4; ++e) xo[j][e] = fmaxf(__fadd_rn(acc[e], b[j][e]), 0.f);
    }
    lstm_wait_vm<0>();        // chunks 0-2 landed
#pragma unroll
    for (int j = 0; j < XRJ; ++j) {
      const int idx = tid + LT * j, row = idx >> 6, c4 = idx & 63;
      *reinterpret_cast<xf4*>(S + 4 * (LSTAGE4 * (c4 >> 5) + (LBN + row) * LLD + (c4 & 31))) = xo[j];
    }
    lstm_lds_barrier();       // chunks 0-2 and every wave's x rows in LDS
    compute(0, accx);
    lstm_lds_barrier();       // everyone is done with stage 0
    issue(3);                 // -> stage 0
    compute(1, accx);
  } else {
    issue(0);
    issue(1);
    issue(2);
    // outstanding per wave after issuing chunks 0..2: 3 LPW
    lstm_wait_vm<2 * LPW>();  // chunk 0 landed (1, 2 in flight)
    lstm_lds_barrier();
    compute(0, accx);
    lstm_wait_vm<LPW>();      // chunk 1 landed (2 in flight)
    lstm_lds_barrier();       // also: everyone is done with stage 0
    issue(3);                 // -> stage 0
    compute(1, accx);
    lstm_wait_vm<LPW>();      // chunk 2 landed (3 in flight)
  }
  lstm_lds_barrier();
  compute(2, acch);
  lstm_wait_vm<0>();          // chunk 3 landed
  lstm_lds_barrier();
  compute(3, acch);

  // ---- epilogue tile into stage 1 (free since the barrier before chunk 2):
  // C row q*4 + r, column col of sub-tile (ms, ns)
  // Chainer's order (a3c_ale.py:50-51, L.LSTM): upward(x) = x Wu^T + b first, then + lateral(h) = h Wl^T
  // (a reset row's state is None: no lateral term)
  float* T = S + 4 * LSTAGE4;
  const float bcol = a.b[n0 + ns * 16 + col];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float up = __fadd_rn(accx[r], bcol);
    T[(ms * 16 + q * 4 + r) * TLD + ns * 16 + col] = rs[r] ? up : __fadd_rn(up, acch[r]);
  }
  if constexpr (XRED) {
    if (n0 == 0) {   // hfc for the backward, from the column-tile-0 workgroups
#pragma unroll
      for (int j = 0; j < XRJ; ++j) {
        const int idx = tid + LT * j, row = idx >> 6, c4 = idx & 63;
        if (m0 + row < a.n) *reinterpret_cast<xf4*>(a.hfc + (int64_t)(m0 + row) * HID + 4 * c4) = xo[j];
      }
    }
  }
  lstm_lds_barrier();
  const int row = tid >> 4, u = tid & 15, m = m0 + row, n = n0 + 4 * u;
  if (m >= a.n) return;
  const float4 g = *reinterpret_cast<const float4*>(T + row * TLD + 4 * u);   // bias added above
  {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{g.x, g.y, g.z, g.w}, reinterpret_cast<f4v*>(a.gates + (int64_t)m * GATES + n));
  }
  if (!a.cell) return;
  const int64_t i = (int64_t)m * HID + (n >> 2);
  const float ag = tanhf(g.x), ig = lstm_sigm(g.y), fg = lstm_sigm(g.z), og = lstm_sigm(g.w);
  const float cp = a.reset[m] ? 0.f : a.c_prev[i];
  const float c = __fadd_rn(__fmul_rn(ag, ig), __fmul_rn(fg, cp));
  a.c_out[i] = c;
  a.h_out[i] = __fmul_rn(og, tanhf(c));
}

hipError_t launch_lstm_gates(const float* x, const float* h, const uint8_t* reset, const float* Wu, const float* Wl,
                             const float* b, float* gates, const float* c_prev, float* c_out, float* h_out, int n,
                             bool cell, hipStream_t s, const float* fc_slab, const float* fc_b, float* hfc) {
  if (n <= 0) return hipSuccess;
  const LstmGatesArgs a{x, h, reset, Wu, Wl, b, gates, c_prev, c_out, h_out, fc_slab, fc_b, hfc, n, cell ? 1 : 0};
  const unsigned blocks = (unsigned)(((n + LBM - 1) / LBM) * (GATES / LBN));
  if (fc_slab != nullptr) {
    if (fc_b == nullptr || hfc == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lstm_gates_kernel<true>, dim3(blocks), dim3(LT), 0, s, a);
  } else {
    if (x == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lstm_gates_kernel<false>, dim3(blocks), dim3(LT), 0, s, a);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Truncated BPTT step of the LSTM backward (a3c.py:129-130 through Chainer
// F.lstm; unchain_backward at the window edge, a3c_ale.py:68-70), one launch
// per step t >= 1:
//
//   dh[m][u]  = sum_j dG_t[m][j] Wl[j][u]        (the lateral Linear's input gradient)
//   dh[m][u]  = 0 where the env reset at step t   (h_{t-1} was None, a3c.py:166)
//   cell = 1: F.lstm backward of step t-1 for (m, u) with dh + dH_{t-1} (the
//             heads' share): dG_{t-1} (4 interleaved gates) and the carried dc
//             -- lstm_cell_bwd_elem's arithmetic (net.hip), op for op;
//   cell = 0: dhn[m][u] = dh only (the split path's separate cell launch reads it).
//
// M = n envs, N = 256 units, K = 1024 gates.  32 x 32 tile per 512-thread
// workgroup; 8 waves = 4 sub-tiles of 16 x 16 x 2 K halves (exact f32
// v_mfma_f32_16x16x4_f32), the halves summed in a fixed order in LDS.  K is
// staged by LDS-DMA in eight 128-column chunks through four LDS stages (three
// chunks in flight, one barrier a chunk): dG_t rows (row stride 33 float4)
// and Wl rows j (32 units + a pad float4, read one float per lane).  The
// epilogue's operands are loaded before the K loop.
namespace {
constexpr int BBM = 32, BBN = 32, BT = 512, BW = BT / 64;
constexpr int BKC = 128;                                 // K chunk
constexpr int BNCH = GATES / BKC;                        // 8 chunks
constexpr int BA_LD = LSTM_LD;                       // 34 float4 per dG row
constexpr int BB_LD = BBN / 4 + 1;                       // 9 float4 per Wl row
constexpr int BA_PC = (BBM * BA_LD + 63) / 64;           // 17 pieces
constexpr int BB_PC = (BKC * BB_LD + 63) / 64;           // 18 pieces
constexpr int BPIECES = BA_PC + BB_PC;                   // 35 pieces a chunk
constexpr int BSTAGE4 = BPIECES * 64;                    // float4 per stage
constexpr int BSTAGES = 4;
constexpr int BTLD = BBN + 4;                            // epilogue half-sum row stride (floats)
static_assert(2 * BBM * BTLD <= BSTAGE4 * 4, "epilogue halves fit one stage");
static_assert(BBM * BBN == 2 * BT, "two (row, unit) pairs per thread");
__host__ __device__ constexpr int bptt_pieces(int w) { return (BPIECES - w + BW - 1) / BW; }
}  // namespace

struct LstmBpttArgs {
  const float* dG;       // (n, 1024) dG_t
  const float* Wl;       // (1024, 256)
  const uint8_t* rs_t;   // (n) reset at step t
  // step t - 1 (cell = 1)
  const float* gates;    // (n, 1024)
  const float* c_t;      // (n, 256) c after step t - 1
  const float* c_prev;   // (n, 256) c before step t - 1
  const uint8_t* rs;     // (n) reset at step t - 1
  const float* dH;       // (n, 256) the heads' dL/dh of step t - 1
  float* dcn;            // (n, 256) carried dc: in from step t, out to step t - 2
  float* dG_out;         // (n, 1024) dG_{t-1}
  float* dhn;            // (n, 256) cell = 0: the masked dh
  int n, cell;
};

__device__ inline void bptt_wait_vm(int n) {   // s_waitcnt vmcnt(n), n wave-uniform
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__global__ void __launch_bounds__(BT)
lstm_bptt_kernel(LstmBpttArgs a) {
  __shared__ __attribute__((aligned(16))) float S[BSTAGES * BSTAGE4 * 4];   // 143,360 B
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NTN = HID / BBN;
  const int m0 = (blockIdx.x / NTN) * BBM, u0 = (blockIdx.x % NTN) * BBN;
  const int pw = bptt_pieces(wave);

  // the epilogue's operands first (the oldest loads: the counted waits cover them)
  int em[2], eu[2];
  float4 eg[2];
  float ec[2], ep[2], eh[2], ed[2];
  uint8_t ers[2], erst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pr = tid + BT * i;              // (row, unit) pair: 32 rows x 32 units
    em[i] = min(m0 + pr / BBN, a.n - 1);
    eu[i] = u0 + pr % BBN;
    const int64_t e = (int64_t)em[i] * HID + eu[i];
    erst[i] = a.rs_t[em[i]];
    if (a.cell) {
      eg[i] = reinterpret_cast<const float4*>(a.gates)[e];
      ec[i] = a.c_t[e];
      ep[i] = a.c_prev[e];
      eh[i] = a.dH[e];
      ed[i] = a.dcn[e];
      ers[i] = a.rs[em[i]];
    }
  }

  auto issue = [&](int c) {
    float* st = S + 4 * BSTAGE4 * (c % BSTAGES);
    const int kc = c * BKC;
    for (int it = wave; it < BPIECES; it += BW) {
      const float* src;
      if (it < BA_PC) {                       // dG_t rows m0.. (rows past n: a valid row, never stored)
        const int i = min(it * 64 + lane, BBM * BA_LD - 1);
        const int r = i / BA_LD, cc = min(i - r * BA_LD, BKC / 4 - 1);
        src = a.dG + (int64_t)min(m0 + r, a.n - 1) * GATES + kc + 4 * cc;
      } else {                                // Wl rows kc.., units u0..u0+31
        const int i = min((it - BA_PC) * 64 + lane, BKC * BB_LD - 1);
        const int r = i / BB_LD, cc = min(i - r * BB_LD, BBN / 4 - 1);
        src = a.Wl + (int64_t)(kc + r) * HID + u0 + 4 * cc;
      }
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + 4 * it * 64), 16, 0, 0);
    }
  };
  issue(0);
  issue(1);
  issue(2);

  const int q = lane >> 4, col = lane & 15;
  const int sub = wave & 3, kh = wave >> 2;   // sub-tile (ms, ns), K half of each chunk
  const int ms = sub & 1, ns = sub >> 1;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < BNCH; ++c) {
    bptt_wait_vm(min(2, BNCH - 1 - c) * pw);  // chunk c landed (up to two later ones in flight)
    lstm_lds_barrier();                       // ... for every wave, and stage (c + 3) % 4 is free
    if (c + 3 < BNCH) issue(c + 3);
    const float* st = S + 4 * BSTAGE4 * (c % BSTAGES);
    const float* Ar = st + (ms * 16 + col) * 4 * BA_LD + 4 * q + 64 * kh;
    const float* Bs = st + 4 * 64 * BA_PC + ns * 16 + col + (64 * kh + 4 * q) * 4 * BB_LD;
    // k = 16 s + 4 q + r of the chunk, s = 4 kh + s4: every fragment of the
    // chunk read first (one LDS wait), then the 16 MFMAs back to back
    f32x4 av[4];
    float bv[4][4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      av[s4] = *reinterpret_cast<const f32x4*>(Ar + 16 * s4);
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[s4][r] = Bs[(16 * s4 + r) * 4 * BB_LD];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s4][r], bv[s4][r], acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  // ---- the two K halves: into stage 0 (free: chunk 4's stage, done two chunks ago), fixed order
  lstm_lds_barrier();
  float* T = S;
#pragma unroll
  for (int r = 0; r < 4; ++r) T[(kh * BBM + ms * 16 + q * 4 + r) * BTLD + ns * 16 + col] = acc[r];
  lstm_lds_barrier();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pr = tid + BT * i, row = pr / BBN, u = pr % BBN;
    if (m0 + row >= a.n) continue;
    float dh = __fadd_rn(T[row * BTLD + u], T[(BBM + row) * BTLD + u]);
    if (erst[i]) dh = 0.f;
    const int64_t e = (int64_t)em[i] * HID + eu[i];
    if (!a.cell) {
      a.dhn[e] = dh;
      continue;
    }
    // lstm_cell_bwd_elem (net.hip) with dh + dH, not first
    const float dht = __fadd_rn(eh[i], dh);
    const float4 g = eg[i];
    const float ag = tanhf(g.x), ig = lstm_sigm(g.y), fg = lstm_sigm(g.z), og = lstm_sigm(g.w);
    const float tc = tanhf(ec[i]);
    float dc = __fmul_rn(__fmul_rn(dht, og), __fsub_rn(1.f, __fmul_rn(tc, tc)));
    dc = __fadd_rn(dc, ed[i]);
    const float cp = ers[i] ? 0.f : ep[i];
    float4 d;
    d.x = __fmul_rn(__fmul_rn(dc, ig), __fsub_rn(1.f, __fmul_rn(ag, ag)));
    d.y = __fmul_rn(__fmul_rn(__fmul_rn(dc, ag), ig), __fsub_rn(1.f, ig));
    d.z = __fmul_rn(__fmul_rn(__fmul_rn(dc, cp), fg), __fsub_rn(1.f, fg));
    d.w = __fmul_rn(__fmul_rn(__fmul_rn(dht, tc), og), __fsub_rn(1.f, og));
    reinterpret_cast<float4*>(a.dG_out)[e] = d;
    a.dcn[e] = ers[i] ? 0.f : __fmul_rn(dc, fg);
  }
}

hipError_t launch_lstm_bptt(const float* dG, const float* Wl, const uint8_t* rs_t, const float* gates, const float* c_t,
                            const float* c_prev, const uint8_t* rs, const float* dH, float* dcn, float* dG_out,
                            float* dhn, int n, bool cell, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const LstmBpttArgs a{dG, Wl, rs_t, gates, c_t, c_prev, rs, dH, dcn, dG_out, dhn, n, cell ? 1 : 0};
  const unsigned blocks = (unsigned)(((n + BBM - 1) / BBM) * (HID / BBN));
  hipLaunchKernelGGL(lstm_bptt_kernel, dim3(blocks), dim3(BT), 0, s, a);
  return hipGetLastError();
}

}  // namespace arl
