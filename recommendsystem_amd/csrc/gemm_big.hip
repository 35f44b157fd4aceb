// Large fp32 GEMMs of the MLP towers (the Dense layers of >= 2^29 multiply-adds, forwards with K >= 1024 from 2^25: the config-3
// trunk and experts, the config-5 experts, the 400-bin head and the DSSM teacher; reference call
// sites staytime/VideoDnn.py:130-148,168-169, rank/multi_head/multidnn.py:80-92,
// rough_rank/model.py:24-27).  Hand-written for gfx950; replaces the round-5 hipBLASLt route.
//
// One kernel template serves the three products of a Dense layer (C[Mo, No] = sum_r A(m, r) B(r, n)):
//   FWD     Y   = act(X W + b)     A = X  [m][r]  (R: contiguous along the reduction)
//                                  B = W  [r][n]  (X: contiguous along the output)
//   DATA    dX (+)= dZ W^T         A = dZ [m][r]  (R, Z operand)   B(r, n) = W[n][r]  (R)
//   WEIGHT  dW (+)= X^T dZ         A(m, r) = X[r][m]  (X)          B = dZ [r][n]      (X, Z operand)
//           db (+)= colsum dZ      as output row K of the same product: A(K, r) = 1 (the "ones
//                                  row" is loaded from a constant, so db costs no extra pass)
// Z operands are dZ = dY act'(Y): the dY and Y tiles both land in LDS and the activation
// derivative is applied to the MFMA fragments as they are read (no dZ pass, no dZ in HBM).
//
// Block = 256 threads (2 x 2 waves), tile BM x BN in {64, 128}^2, reduction slabs of BK = 16 in a
// STAGES-deep LDS ring filled by direct-to-LDS DMA (global_load_lds_dwordx4, or _dword for
// operands whose rows are not 16-B aligned): no VGPR round trip, the next STAGES - 1 slabs in
// flight while one feeds the MFMAs, one LDS-only barrier per slab.  Images:
//   R operand: [x][16] rows, 16-B chunks XOR-swizzled by sw_r(x) so the float4 fragment reads of a
//              16-row tile hit 16 distinct bank quads in each ds_read_b128 lane group; a lane's
//              float4 covers four k-steps of v_mfma_f32_16x16x4_f32 (k permuted identically in A
//              and B: k-step t of lane group q takes r = 4q + t);
//   X operand: [r][BX] rows (the global rows as they are), chunks XOR-swizzled by sw_x(r) so the
//              four lane groups' rows of one ds_read_b32 land in different 16-bank quarters.
// Split-K (deterministic): per-split partial slabs + the fixed-order column reduce of dense.hip.
// Tile order: blocks b and b + 8 share an XCD (and its L2), so the grid is re-indexed to give
// each XCD a contiguous range of tiles, grouped GM tile rows at a time (A and B panels reused
// from that XCD's L2).
#include "gemm_big.hpp"

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

namespace rs_big {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16-B aligned constants: zeros (the reduction tail / padding) and ones (the db row)
__device__ __attribute__((aligned(16))) float g_consts[8] = {0.f, 0.f, 0.f, 0.f, 1.f, 1.f, 1.f, 1.f};

constexpr int BK = 16;
// waves per block (tuning knob): 4 = one per SIMD, 8 = two per SIMD (one stalls, the other
// feeds the matrix pipe)
#ifndef RS_BIG_NW
#define RS_BIG_NW 4
#endif
constexpr int NW = RS_BIG_NW;
constexpr int kThreads = 64 * NW;
// tuning knobs (compile-time): 16-deep slabs per pipeline stage (one barrier per stage) and the
// ring depth without / with a Z operand
#ifndef RS_BIG_KSUB
#define RS_BIG_KSUB 1
#endif
#ifndef RS_BIG_STAGES_NZ
#define RS_BIG_STAGES_NZ 4
#endif
#ifndef RS_BIG_STAGES_Z
#define RS_BIG_STAGES_Z 3
#endif
#ifndef RS_BIG_INTERLEAVE
#define RS_BIG_INTERLEAVE 1
#endif
constexpr int KSUB = RS_BIG_KSUB;

// R image: slot of chunk c of tile row x is c ^ sw_r(x); sw_r over (x >> 2) & 3 = {0, 2, 3, 1}
// makes the (q, j) lanes of each ds_read_b128 group (lanes {0-3, 12-15, 20-27}, ...) distinct
__host__ __device__ constexpr int sw_r(int x) { return (0x1320 >> (4 * ((x >> 2) & 3))) & 3; }
// X image: slot of chunk c of reduction row r is c ^ sw_x(r): lane group q = r >> 2 moves by 16
// floats (rows of >= 64 floats: the four groups of a ds_read_b32 in four 16-bank quarters); a
// 32-float row holds 8 chunks, so there the XOR stays below 8 (groups 0 / 1 and 2 / 3 apart,
// the pairs that share a lane half of the instruction)
template <int BX>
__host__ __device__ constexpr int sw_x(int r) {
  return BX >= 64 ? ((r >> 2) & 3) << 2 : ((r >> 2) & 1) << 2;
}

enum { MODE_R = 0, MODE_X = 1 };

__device__ __forceinline__ float act_fwd(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return 1.0f / (1.0f + expf(-v));
  return v;
}
__device__ __forceinline__ float act_bwd(float dy, float y, int act) {
  if (act == 1) return y > 0.f ? dy : 0.f;
  if (act == 2) return dy * y * (1.0f - y);
  return dy;
}

__device__ __forceinline__ void dma16(uint32_t lds, const float* g) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void dma4(uint32_t lds, const float* g) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the DMAs are invisible to the compiler's counters)
__device__ __forceinline__ void vm_wait_n(int n) {
#define RS_W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    RS_W(0) RS_W(1) RS_W(2) RS_W(3) RS_W(4) RS_W(5) RS_W(6) RS_W(7) RS_W(8) RS_W(9) RS_W(10)
    RS_W(11) RS_W(12) RS_W(13) RS_W(14) RS_W(15) RS_W(16) RS_W(17) RS_W(18) RS_W(19) RS_W(20)
    RS_W(21) RS_W(22) RS_W(23) RS_W(24) RS_W(25) RS_W(26) RS_W(27) RS_W(28) RS_W(29) RS_W(30)
    RS_W(31) RS_W(32) RS_W(33) RS_W(34) RS_W(35) RS_W(36) RS_W(37) RS_W(38) RS_W(39) RS_W(40)
    RS_W(41) RS_W(42) RS_W(43) RS_W(44) RS_W(45) RS_W(46) RS_W(47) RS_W(48) RS_W(49) RS_W(50)
    RS_W(51) RS_W(52) RS_W(53) RS_W(54) RS_W(55) RS_W(56) RS_W(57) RS_W(58) RS_W(59) RS_W(60)
    RS_W(61) RS_W(62)
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
#undef RS_W
}

__device__ __forceinline__ void lds_sync() {
#ifdef RS_BIG_NOBAR  // diagnostic builds only (with RS_BIG_NODMA): the barrier's share
  return;
#endif
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ uint32_t lds_off(const float* p) {
  uint32_t v = (uint32_t)(uintptr_t)p;
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}

// DMA of one operand slab: tile rows [x0, x0 + BX) x reduction [r0, r0 + BK) into the image at
// dst (BX * BK floats).  Each lane's addresses are computed once (init) and advanced by one slab
// per issue; rows past X read row X - 1 (their products land in output rows / columns that are
// never stored) -- except the ones row (x == X with ones set) of the WEIGHT A operand; in the
// last slab of a split (tail) reduction indices at or past re read zeros.  IPW instructions per
// wave (uniform).
template <int BX, int MODE, bool VEC_>
struct OpDma {
  static constexpr int FL = BX * BK;
  // 16-B pieces when they split evenly over the waves (otherwise 4-B pieces)
  static constexpr bool VEC = VEC_ && (FL / 4 / 64) % NW == 0;
  static constexpr int IPW = VEC ? FL / 4 / 64 / NW : FL / 64 / NW;
  static_assert(IPW >= 1, "tile too small");
  const float* cur[IPW];
  int rl[IPW];
  bool one[IPW];
  int64_t step;

  __device__ void init(const float* p, int64_t ld, int64_t x0, int64_t X, int ones, int64_t rb,
                       int w, int lane) {
    step = MODE == MODE_R ? BK : BK * ld;
#pragma unroll
    for (int u = 0; u < IPW; ++u) {
      const int i = w * IPW + u;
      int64_t x;
      int r;
      if constexpr (VEC) {
        const int c = 64 * i + lane;
        if constexpr (MODE == MODE_R) {
          const int row = c >> 2;
          x = x0 + row;
          r = 4 * ((c & 3) ^ sw_r(row));
        } else {
          constexpr int CPR = BX / 4;
          const int row = c / CPR;
          r = row;
          x = x0 + 4 * ((c % CPR) ^ sw_x<BX>(row));
        }
      } else {
        const int d = 64 * i + lane;
        if constexpr (MODE == MODE_R) {
          const int row = d >> 4, wi = d & 15;
          x = x0 + row;
          r = 4 * ((wi >> 2) ^ sw_r(row)) + (wi & 3);
        } else {
          const int row = d / BX, wi = d % BX;
          r = row;
          x = x0 + 4 * ((wi >> 2) ^ sw_x<BX>(row)) + (wi & 3);
        }
      }
      one[u] = ones && x == X;
      if (x >= X) x = VEC && MODE == MODE_X ? X - 4 : X - 1;  // (VEC X rows: X % 4 == 0)
      rl[u] = r;
      cur[u] = p + (MODE == MODE_R ? x * ld + rb + r : (rb + r) * ld + x);
    }
  }
  // issue the next slab (starting at reduction index r0) into the image at dst
  __device__ void issue(float* dst, int64_t r0, int64_t re, bool tail) {
#ifdef RS_BIG_NODMA  // diagnostic builds only: the MFMA / LDS pipeline without its loads
    return;
#endif
#pragma unroll
    for (int u = 0; u < IPW; ++u) {
      const float* g = one[u] ? g_consts + 4 : cur[u];
      if (tail && r0 + rl[u] >= re) g = g_consts;
      if constexpr (VEC) dma16(lds_off(dst + 256 * (threadIdx.x / 64 * IPW + u)), g);
      else dma4(lds_off(dst + 64 * (threadIdx.x / 64 * IPW + u)), g);
      cur[u] += step;
    }
  }
};

// (the counter holds 63 at most: a larger allowance waits for a little more than needed)
template <int N>
__device__ __forceinline__ void vm_wait_c() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N > 63 ? 63 : N) : "memory");
}

// fragments of one slab: A rows / B columns of this wave, four k-steps each
template <int TMW, int TNW>
struct Frag {
  float a[TMW][4], b[TNW][4];
};

// WM x WN waves (NW in all); wave tile (BM / WM) x (BN / WN)
template <int BM, int BN>
struct WaveGrid {
  static constexpr int WN = BN >= 64 ? 2 : 1;
  static constexpr int WM = NW / WN;
  static constexpr int TMW = BM / WM / 16, TNW = BN / WN / 16;
  static_assert(TMW >= 1 && TNW >= 1, "wave tile");
};

template <int BM, int BN, int AMODE, int BMODE, bool AVEC, bool BVEC, bool ZA, bool ZB>
__global__ void __launch_bounds__(kThreads, NW == 8 ? 1 : 2) big_kernel(Args g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  using DA = OpDma<BM, AMODE, AVEC>;
  using DB = OpDma<BN, BMODE, BVEC>;
  using WG = WaveGrid<BM, BN>;
  constexpr int TMW = WG::TMW, TNW = WG::TNW;
  constexpr int STAGES = (ZA || ZB) ? RS_BIG_STAGES_Z : RS_BIG_STAGES_NZ;
  constexpr int IPS = KSUB * (DA::IPW * (ZA ? 2 : 1) + DB::IPW * (ZB ? 2 : 1));
  // per-slab image: A | B | A's Y | B's Y; a stage holds KSUB slabs
  constexpr int SB = DA::FL, SAY = SB + DB::FL, SBY = SAY + (ZA ? DA::FL : 0);
  constexpr int SFL1 = SBY + (ZB ? DB::FL : 0);
  constexpr int SFL = KSUB * SFL1;
  constexpr int KST = KSUB * BK;  // reduction rows per stage
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int q = lane >> 4, j = lane & 15;
  const int wr = w / WG::WN, wc = w % WG::WN;

  // ---- block -> (split, tile): XCD-contiguous ranges, GM tile rows per group ----
  const int nb = (int)gridDim.x;
  int b = (int)blockIdx.x;
  if (g.xcd && (nb & 7) == 0) b = (b & 7) * (nb >> 3) + (b >> 3);
  const int T = g.tm * g.tn;
  const int z = b / T, tt = b - z * T;
  const int per_group = g.gm * g.tn;
  const int grp = tt / per_group, first = grp * g.gm;
  const int gsz = (g.tm - first) < g.gm ? (g.tm - first) : g.gm;
  const int within = tt - grp * per_group;
  const int tm = first + within % gsz, tn = within / gsz;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t rb = (int64_t)z * g.rchunk;
  const int64_t re = rb + g.rchunk < g.R ? rb + g.rchunk : g.R;
  const int nst = (int)((re - rb + KST - 1) / KST);

  DA da, day;
  DB db, dby;
  da.init(g.a.p, g.a.ld, m0, g.a.X, g.a.ones, rb, w, lane);
  db.init(g.b.p, g.b.ld, n0, g.b.X, 0, rb, w, lane);
  if constexpr (ZA) day.init(g.a.y, g.a.ldy, m0, g.a.X, 0, rb, w, lane);
  if constexpr (ZB) dby.init(g.b.y, g.b.ldy, n0, g.b.X, 0, rb, w, lane);
  auto issue = [&](int s) {
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub) {
      float* st = smem + (s % STAGES) * SFL + sub * SFL1;
      const int64_t r0 = rb + (int64_t)s * KST + sub * BK;
      const bool tail = r0 + BK > re;
      da.issue(st, r0, re, tail);
      db.issue(st + SB, r0, re, tail);
      if constexpr (ZA) day.issue(st + SAY, r0, re, tail);
      if constexpr (ZB) dby.issue(st + SBY, r0, re, tail);
    }
  };
  // fragment reads of slab s (Z operands: dY raw into the fragment, Y beside it)
  auto read1 = [&](const float* st, Frag<TMW, TNW>& f, Frag<ZA ? TMW : 1, ZB ? TNW : 1>& fy) {
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const int x = wr * (BM / WG::WM) + 16 * i + j;
      if constexpr (AMODE == MODE_R) {
        const int o = x * BK + 4 * (q ^ sw_r(x));
        const float4 v = *reinterpret_cast<const float4*>(st + o);
        f.a[i][0] = v.x; f.a[i][1] = v.y; f.a[i][2] = v.z; f.a[i][3] = v.w;
        if constexpr (ZA) {
          const float4 y = *reinterpret_cast<const float4*>(st + SAY + o);
          fy.a[i][0] = y.x; fy.a[i][1] = y.y; fy.a[i][2] = y.z; fy.a[i][3] = y.w;
        }
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = 4 * q + u;
          const int o = r * BM + 4 * ((x >> 2) ^ sw_x<BM>(r)) + (x & 3);
          f.a[i][u] = st[o];
          if constexpr (ZA) fy.a[i][u] = st[SAY + o];
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < TNW; ++jj) {
      const int x = wc * (BN / WG::WN) + 16 * jj + j;
#ifdef RS_BIG_DIAG_BR  // diagnostic builds only: B fragments read as R images (wrong values)
      if constexpr (true) {
#else
      if constexpr (BMODE == MODE_R) {
#endif
        const int o = x * BK + 4 * (q ^ sw_r(x));
        const float4 v = *reinterpret_cast<const float4*>(st + SB + o);
        f.b[jj][0] = v.x; f.b[jj][1] = v.y; f.b[jj][2] = v.z; f.b[jj][3] = v.w;
        if constexpr (ZB) {
          const float4 y = *reinterpret_cast<const float4*>(st + SBY + o);
          fy.b[jj][0] = y.x; fy.b[jj][1] = y.y; fy.b[jj][2] = y.z; fy.b[jj][3] = y.w;
        }
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = 4 * q + u;
          const int o = r * BN + 4 * ((x >> 2) ^ sw_x<BN>(r)) + (x & 3);
          f.b[jj][u] = st[SB + o];
          if constexpr (ZB) fy.b[jj][u] = st[SBY + o];
        }
      }
    }
  };
  using FY = Frag<ZA ? TMW : 1, ZB ? TNW : 1>;
  auto read = [&](int s, Frag<TMW, TNW> (&f)[KSUB], FY (&fy)[KSUB]) {
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub) read1(smem + (s % STAGES) * SFL + sub * SFL1, f[sub], fy[sub]);
  };
  auto zform1 = [&](Frag<TMW, TNW>& f, const Frag<ZA ? TMW : 1, ZB ? TNW : 1>& fy) {
    if constexpr (ZA) {
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int u = 0; u < 4; ++u) f.a[i][u] = act_bwd(f.a[i][u], fy.a[i][u], g.act_z);
    }
    if constexpr (ZB) {
#pragma unroll
      for (int jj = 0; jj < TNW; ++jj)
#pragma unroll
        for (int u = 0; u < 4; ++u) f.b[jj][u] = act_bwd(f.b[jj][u], fy.b[jj][u], g.act_z);
    }
  };

  f32x4 acc[TMW][TNW];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int jj = 0; jj < TNW; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto zform = [&](Frag<TMW, TNW> (&f)[KSUB], const FY (&fy)[KSUB]) {
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub) zform1(f[sub], fy[sub]);
  };
  auto mma = [&](const Frag<TMW, TNW> (&fs)[KSUB]) {
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub)
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
          for (int jj = 0; jj < TNW; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(fs[sub].a[i][u], fs[sub].b[jj][u],
                                                              acc[i][jj], 0, 0, 0);
  };

  // ---- pipeline: STAGES slabs in flight; slab s + 1's fragments are read while slab s's MFMAs
  // run (its slot is refilled once every wave has passed the next barrier) ----
  const int pro = nst < STAGES ? nst : STAGES;
  for (int s = 0; s < pro; ++s) issue(s);
  Frag<TMW, TNW> f0[KSUB], f1[KSUB];
  FY y0[KSUB], y1[KSUB];
  vm_wait_n(IPS * (pro - 1));
  lds_sync();
  read(0, f0, y0);
  zform(f0, y0);
  // One slab step.  STEADY (slab s + STAGES exists): a constant wait count, the next DMA issued
  // and slab s + 1's fragments read unconditionally -- no branch in front of the MFMAs (behind a
  // conditional read the compiler's wait pass put an lgkmcnt(0) there, which waited for those
  // reads before this slab's MFMAs).  The tail steps (the last STAGES or so) count exactly.
  auto mma_issue = [&](int s, Frag<TMW, TNW> (&fc)[KSUB], bool iss) {
#if RS_BIG_INTERLEAVE
    // the next DMA pieces issued between the k-step groups of this slab's MFMAs (one wave per
    // SIMD issues in order: a block of address VALU + DMA in front of the MFMAs would not
    // overlap them)
    constexpr int NPO = 2 + (ZA ? 1 : 0) + (ZB ? 1 : 0);  // pieces per slab
#pragma unroll
    for (int sub = 0; sub < KSUB; ++sub)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
          for (int jj = 0; jj < TNW; ++jj)
#ifdef RS_BIG_NOMFMA  // diagnostic builds only: the load pipeline without its MFMAs
            acc[i][jj][0] += fc[sub].a[i][u] * fc[sub].b[jj][u];
#else
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(fc[sub].a[i][u], fc[sub].b[jj][u],
                                                              acc[i][jj], 0, 0, 0);
#endif
        __builtin_amdgcn_sched_barrier(0);
        if (iss && u < NPO) {
          const int s2 = s + STAGES;
          float* st = smem + (s2 % STAGES) * SFL + sub * SFL1;
          const int64_t r0 = rb + (int64_t)s2 * KST + sub * BK;
          const bool tail = r0 + BK > re;
          if (u == 0) da.issue(st, r0, re, tail);
          else if (u == 1) db.issue(st + SB, r0, re, tail);
          else if (u == 2 && ZA) day.issue(st + SAY, r0, re, tail);
          else if constexpr (ZB) dby.issue(st + SBY, r0, re, tail);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#else
    if (iss) issue(s + STAGES);
    mma(fc);
#endif
  };
  auto steady = [&](int s, Frag<TMW, TNW> (&fc)[KSUB], Frag<TMW, TNW> (&fn)[KSUB], FY (&yn)[KSUB]) {
    vm_wait_c<IPS * (STAGES - 2)>();  // slab s + 1 landed (this wave's DMAs)
    lds_sync();                        // ... every wave's; slot s free
    read(s + 1, fn, yn);
    mma_issue(s, fc, true);
    zform(fn, yn);
  };
  auto tail_step = [&](int s, Frag<TMW, TNW> (&fc)[KSUB], Frag<TMW, TNW> (&fn)[KSUB], FY (&yn)[KSUB]) {
    const bool more = s + 1 < nst;
    const int issued = s + STAGES < nst ? s + STAGES : nst;
    if (more) vm_wait_n(IPS * (issued - s - 2));
    lds_sync();
    if (more) read(s + 1, fn, yn);
    mma_issue(s, fc, s + STAGES < nst);
    if (more) zform(fn, yn);
  };
  int s = 0;
  for (; s + 1 + STAGES < nst; s += 2) {
    steady(s, f0, f1, y1);
    steady(s + 1, f1, f0, y0);
  }
  for (; s < nst; s += 2) {
    tail_step(s, f0, f1, y1);
    if (s + 1 < nst) tail_step(s + 1, f1, f0, y0);
  }

  // ---- epilogue: lane (q, j) holds C[16-row tile + 4q + rr][16-col tile + j] ----
  // (every load of the accumulating / bias forms is issued before the first store)
  float prev[TMW][TNW][4];
  const bool acc_in = g.epi == EPI_STORE && g.accumulate;
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int jj = 0; jj < TNW; ++jj) {
      const int64_t n = n0 + wc * (BN / WG::WN) + 16 * jj + j;
      const bool nok = n < g.N;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int64_t m = m0 + wr * (BM / WG::WM) + 16 * i + 4 * q + rr;
        float v = 0.f;
        if (g.epi == EPI_FWD) {
          v = nok ? g.bias[n] : 0.f;
        } else if (acc_in && nok) {
          if (m < g.Mreal) v = g.out[m * g.ldo + n];
          else if (m == g.Mreal && g.db) v = g.db[n];
        }
        prev[i][jj][rr] = v;
      }
    }
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int jj = 0; jj < TNW; ++jj) {
      const int64_t n = n0 + wc * (BN / WG::WN) + 16 * jj + j;
      if (n >= g.N) continue;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int64_t m = m0 + wr * (BM / WG::WM) + 16 * i + 4 * q + rr;
        const float v = acc[i][jj][rr] + prev[i][jj][rr];
        if (g.epi == EPI_FWD) {
          if (m < g.M) g.out[m * g.ldo + n] = act_fwd(v, g.act);
        } else if (g.epi == EPI_STORE) {
          if (m < g.Mreal) g.out[m * g.ldo + n] = v;
          else if (m == g.Mreal && g.db) g.db[n] = v;
        } else {
          if (m < g.M) g.out[(int64_t)z * g.slab + m * g.N + n] = acc[i][jj][rr];
        }
      }
    }
}

// split-K forward: the splits' partial [M, N] slabs summed in split order, + bias, activation
__global__ void __launch_bounds__(256) fwd_reduce_kernel(const float* __restrict__ part, int splits,
                                                         int64_t M, int64_t N,
                                                         const float* __restrict__ bias, int act,
                                                         float* __restrict__ out, int64_t ldo) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= M * N) return;
  const int64_t m = k / N, n = k - m * N;
  float v = part[k];
  for (int s = 1; s < splits; ++s) v += part[(int64_t)s * M * N + k];
  out[m * ldo + n] = act_fwd(v + bias[n], act);
}

// ---------------------------------------------------------------------------------------------
struct Tile { int bm, bn; };

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

static int stages_of(bool z) { return z ? RS_BIG_STAGES_Z : RS_BIG_STAGES_NZ; }

size_t lds_bytes(int bm, int bn, bool za, bool zb) {
  return (size_t)stages_of(za || zb) * KSUB *
         ((size_t)bm * BK * (za ? 2 : 1) + (size_t)bn * BK * (zb ? 2 : 1)) * 4;
}

// Tile / split choice: the multiply-adds of the busiest CU (blocks per CU share its matrix
// pipes) at the rate the kernel reaches on a busy CU, plus a split-K's partial round trip and
// reduce launch; larger tiles win ties (fewer operand bytes per flop).  The constants are fitted
// to a forced tile x split sweep of the configs 3 / 5 trunk shapes (profiles/r06/gemm/
// tile_sweep.txt): ~150 k MAC/us per busy CU whatever the tile (~49 % of the f32 MFMA peak), a
// 64 x 64 tile ~10 % above that (4 blocks per CU: two waves per SIMD hide the LDS / barrier
// waits), a split ~6 us + its partial slabs at ~4 TB/s.  (The round-5 form priced the tiles at
// the MFMA peak with 64 x 64 at 0.75 and picked 128-row tiles 1 per CU: 10-35 % slower on 6 of
// the 9 trunk products.)  RS_GEMM_BIG_TILE=BMxBN[,S] forces a choice (tuning runs).
Plan plan(int64_t M, int64_t N, int64_t R, bool allow_split, bool z) {
  static const Tile cand[4] = {{128, 128}, {128, 64}, {64, 64}, {128, 32}};
  // (N <= 32: the 128 x 32 tile first -- it pads the outputs to 32 columns, not 64, so at equal
  // modelled cost it does half the MFMA work: 2048 x 1456 x 22 forward 16.0 -> 14.8 us)
  static const Tile cand_narrow[4] = {{128, 32}, {128, 128}, {128, 64}, {64, 64}};
  const Tile* cands = N <= 32 ? cand_narrow : cand;
  Plan best{};
  double bc = 0;
  for (int c = 0; c < 4; ++c) {
    const int bm = cands[c].bm, bn = cands[c].bn;
    if (bn == 32 && N > 32) continue;
    const int64_t tiles = cdiv(M, bm) * cdiv(N, bn);
    for (int64_t s = 1; s <= (allow_split ? 16 : 1); s *= 2) {
      if (s > 1 && (R / s < 128 || tiles * s > 1536)) break;
      const int64_t rc = cdiv(cdiv(R, s), BK) * BK;
      const int64_t blocks = tiles * cdiv(R, rc);
      const double per_cu = (double)cdiv(blocks, 256);
      const double rate = 150000.0 * (bm * bn <= 4096 ? 1.1 : 1.0);  // MAC per us per CU
      double cost = per_cu * (double)bm * bn * rc / rate;
      if (s > 1) cost += (double)s * M * N * 8.0 / 4.0e6 + 6.0;
      if (best.bm == 0 || cost < bc * 0.98) {
        bc = cost;
        best = Plan{bm, bn, (int)cdiv(R, rc), rc, stages_of(z)};
      }
    }
  }
  // Outputs just past a multiple of 64 columns (config 3's N = 273): 128 x 32 tiles trim >= 10 %
  // of the padded columns; split so the grid holds ~4 blocks per CU (<= 1536 blocks) -- measured
  // best of each product's tile x split sweep (forward 4096 x 1616 x 273 71.3 -> 66.9 us, weight
  // 89.8 -> 73.6 us; profiles/r06/gemm/tile_n273.txt).  The model above ties these tiles (both pad
  // their work to the same per-CU count) and under-prices the 4-B DMA path at one block per CU.
  if (allow_split && N > 32 && cdiv(N, 32) * 32 * 10 <= cdiv(N, 64) * 64 * 9) {
    const int64_t tiles = cdiv(M, 128) * cdiv(N, 32);
    int64_t s = 1;
    while (s < 16 && tiles * s * 2 <= 1536 && R / (s * 2) >= 128) s *= 2;
    const int64_t rc = cdiv(cdiv(R, s), BK) * BK;
    best = Plan{128, 32, (int)cdiv(R, rc), rc, stages_of(z)};
  }
  static const int forced = [] {
    const char* e = getenv("RS_GEMM_BIG_TILE");
    int bm = 0, bn = 0, s = 0;
    if (e && sscanf(e, "%dx%d,%d", &bm, &bn, &s) >= 2) return bm * 100000 + bn * 100 + s;
    return 0;
  }();
  if (forced) {
    best.bm = forced / 100000;
    best.bn = (forced / 100) % 1000;
    int s = forced % 100;
    if (!allow_split || s < 1) s = 1;
    best.rchunk = cdiv(cdiv(R, s), BK) * BK;
    best.splits = (int)cdiv(R, best.rchunk);
    best.stages = stages_of(z);
  }
  return best;
}

template <int AMODE, int BMODE, bool AV, bool BV, bool ZA, bool ZB>
static int launch_t(hipStream_t s, const Plan& p, Args g) {
  g.tm = (int)cdiv(g.M, p.bm);
  g.tn = (int)cdiv(g.N, p.bn);
  static const int gm = [] {  // tile rows per group (tuning: RS_GEMM_BIG_GM; 0 = no XCD remap)
    const char* e = getenv("RS_GEMM_BIG_GM");
    return e ? atoi(e) : 4;
  }();
  g.gm = gm > 0 ? gm : 1;
  g.xcd = gm > 0;
  g.rchunk = p.rchunk;
  const int64_t blocks = (int64_t)g.tm * g.tn * p.splits;
  if (blocks <= 0 || blocks > (1 << 30)) return 1;
  const size_t lds = lds_bytes(p.bm, p.bn, ZA, ZB);
#define RS_BIG(BM_, BN_) \
  big_kernel<BM_, BN_, AMODE, BMODE, AV, BV, ZA, ZB><<<(unsigned)blocks, kThreads, lds, s>>>(g)
  if (p.bm == 128 && p.bn == 128) RS_BIG(128, 128);
  else if (p.bm == 128 && p.bn == 64) RS_BIG(128, 64);
  else if (p.bm == 64 && p.bn == 64) RS_BIG(64, 64);
  else if (p.bm == 128 && p.bn == 32) RS_BIG(128, 32);
  else return 1;
#undef RS_BIG
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// VEC (16-B DMA pieces) for an operand whose rows start 16-B aligned and whose contiguous extent
// splits into whole chunks: R operands along the reduction (R % 4), X operands along the output
// (X % 4; the ones row needs X % 4 == 0 too, it is one whole chunk)
int launch(hipStream_t s, int form, const Plan& p, const Args& g) {
  const bool za = g.a.y != nullptr, zb = g.b.y != nullptr;
  const bool av = al16(g.a.p) && (!za || (al16(g.a.y) && g.a.ldy % 4 == 0)) && g.a.ld % 4 == 0 &&
                  (form == FORM_WEIGHT ? g.a.X % 4 == 0 : g.R % 4 == 0);
  const bool bv = al16(g.b.p) && (!zb || (al16(g.b.y) && g.b.ldy % 4 == 0)) && g.b.ld % 4 == 0 &&
                  (form == FORM_DATA ? g.R % 4 == 0 : g.b.X % 4 == 0);
  if (form == FORM_FWD) {
    if (za || zb) return 1;
    if (av && bv) return launch_t<MODE_R, MODE_X, true, true, false, false>(s, p, g);
    if (av) return launch_t<MODE_R, MODE_X, true, false, false, false>(s, p, g);
    if (bv) return launch_t<MODE_R, MODE_X, false, true, false, false>(s, p, g);
    return launch_t<MODE_R, MODE_X, false, false, false, false>(s, p, g);
  }
  if (form == FORM_DATA) {  // A (dY rows) and B (W rows) share the reduction extent N
    if (zb) return 1;
    const bool v = av && bv;
    if (za) return v ? launch_t<MODE_R, MODE_R, true, true, true, false>(s, p, g)
                     : launch_t<MODE_R, MODE_R, false, false, true, false>(s, p, g);
    return v ? launch_t<MODE_R, MODE_R, true, true, false, false>(s, p, g)
             : launch_t<MODE_R, MODE_R, false, false, false, false>(s, p, g);
  }
  if (form == FORM_WEIGHT) {
    if (za) return 1;
#define RS_WF(Z)                                                                 \
    if (av && bv) return launch_t<MODE_X, MODE_X, true, true, false, Z>(s, p, g);   \
    if (av) return launch_t<MODE_X, MODE_X, true, false, false, Z>(s, p, g);        \
    if (bv) return launch_t<MODE_X, MODE_X, false, true, false, Z>(s, p, g);        \
    return launch_t<MODE_X, MODE_X, false, false, false, Z>(s, p, g);
    if (zb) { RS_WF(true) }
    RS_WF(false)
#undef RS_WF
  }
  return 1;
}

// the forward's split-K partials: a process-wide slab per device, grown only outside graph
// capture and never freed (a captured graph keeps the address it was recorded with)
static float* fwd_scratch(size_t floats, hipStream_t s) {
  struct Slab { float* buf = nullptr; size_t cap = 0; std::vector<float*> retired; };
  static std::mutex mu;
  static std::map<int, Slab> slabs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  Slab& sl = slabs[dev];
  if (floats <= sl.cap) return sl.buf;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  size_t want = sl.cap ? 2 * sl.cap : floats;
  if (want < floats) want = floats;
  float* nb = nullptr;
  if (hipMalloc(&nb, want * sizeof(float)) != hipSuccess) return nullptr;
  if (sl.buf) sl.retired.push_back(sl.buf);
  sl.buf = nb;
  sl.cap = want;
  return sl.buf;
}

bool wanted_fwd(int64_t M, int64_t N, int64_t K) {
  static const bool on = [] {
    const char* e = getenv("RS_GEMM_BIG");
    return !e || atoi(e) != 0;
  }();
  // (from 2^25 multiply-adds: config 5's 2048 x 1456 x 22 forward 26.9 us on the engine, 14.8 on
  // these kernels -- a long reduction split over the chip; profiles/r06/gemm/tile_small.txt)
  return wanted(M, N, K) || (on && K >= 1024 && M * N * K >= ((int64_t)1 << 25));
}

int fwd(hipStream_t s, const float* X, int64_t M, int64_t K, int64_t ldx, const float* W,
        const float* bias, int64_t N, int act, float* Y, int64_t ldy) {
  Plan p = plan(M, N, K, true, false);
  float* part = nullptr;
  if (p.splits > 1) {
    part = fwd_scratch((size_t)p.splits * M * N, s);
    if (!part) p = plan(M, N, K, false, false);  // (capturing before an eager call sized it)
  }
  Args g{};
  g.a = Operand{X, nullptr, ldx, 0, M, 0};
  g.b = Operand{W, nullptr, N, 0, N, 0};
  g.M = M; g.N = N; g.R = K; g.Mreal = M;
  if (p.splits > 1) {
    g.epi = EPI_PARTIAL; g.out = part; g.slab = M * N;
  } else {
    g.epi = EPI_FWD; g.act = act; g.bias = bias; g.out = Y; g.ldo = ldy;
  }
  if (launch(s, FORM_FWD, p, g)) return 1;
  if (p.splits > 1)
    fwd_reduce_kernel<<<(unsigned)cdiv(M * N, 256), 256, 0, s>>>(part, p.splits, M, N, bias, act, Y, ldy);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// From 2^29 multiply-adds the big kernels beat the round-4 engine on every configs 3 / 5 product;
// between 2^25 and 2^29 only the forward with a long reduction (>= 1024: split-K fills the
// chip) does -- the short-reduction shapes (2048 x 224 x 1152, 2048 x 528 x 400, 2048 x 832 x
// 128) keep the engine (tools/r06_shapes.sh, profiles/r06/gemm/shapes.txt)
bool wanted(int64_t m, int64_t n, int64_t k) {
  static const int64_t thr = [] {
    const char* e = getenv("RS_GEMM_BIG_MACS");
    return e ? (int64_t)atoll(e) : ((int64_t)1 << 29);
  }();
  static const bool on = [] {
    const char* e = getenv("RS_GEMM_BIG");
    return !e || atoi(e) != 0;
  }();
  return on && m > 0 && n > 0 && k > 0 && m * n * k >= thr;
}

}  // namespace rs_big
