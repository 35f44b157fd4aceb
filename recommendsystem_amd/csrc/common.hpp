// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of the CTR feature-interaction path.
//
// Every exported entry point is a plain C-ABI function (see include/recsys_amd.h): raw device
// pointers, explicit sizes, a hipStream_t passed as void*, an int status.  Nothing here allocates,
// frees or synchronises, so every launch can be captured into a hipGraph by the caller.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define RS_API extern "C" __attribute__((visibility("default")))

enum {
  RS_OK = 0,
  RS_ERR_ARG = -1,          // bad shape / null pointer / inconsistent sizes
  RS_ERR_UNSUPPORTED = -2,  // shape outside the compiled instantiations
  RS_ERR_LAUNCH = -3,       // hipLaunch failed (hipGetLastError != success)
};

static inline int rs_status_after_launch() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? RS_OK : RS_ERR_LAUNCH;
}

static inline hipStream_t rs_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Math mode (rs_set_math_mode, include/recsys_amd.h): process-wide, read when a launch is issued
// (so a captured graph keeps the mode it was captured under).  Process-wide rather than per
// thread because PyTorch's autograd issues the backward launches from its own device thread.
enum { RS_MATH_F32 = 0, RS_MATH_BF16 = 1 };
int rs_math_mode_now();

// Dropout seed offset source (rs_set_seed_offset): a device int64 read by the kernel when it
// runs, so a captured graph replayed step after step draws a new mask each step (the trainers
// point it at their device step counter).  Read at launch, like the math mode.
const int64_t* rs_seed_offset_now();
// off_addr: the device address of the int64 offset, 0 = none (carried as an integer).  The
// load is one scalar load in inline asm, done once at kernel entry: as a plain C++ load
// (generic or global pointer) inside the IL kernels' per-iteration loops it tripped a gfx950
// backend error ("Operand has incorrect register class" on a flat-aperture compare).  Not volatile and no memory clobber: the value is constant for the
// launch, so the compiler may hoist / merge it.
__device__ __forceinline__ uint64_t rs_eff_seed(uint64_t seed, uint64_t off_addr) {
  if (!off_addr) return seed;
  // uniform by construction (a kernel argument); readfirstlane pins it to SGPRs even where
  // register pressure would otherwise leave it in VGPRs ("s" constraint on a VGPR pair)
  const uint64_t sa = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(off_addr >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)off_addr);
  uint64_t v;
  asm("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(sa));
  return seed + v * 0x9E3779B97F4A7C15ull;
}

// bf16 math mode GEMM step.  v_mfma_f32_16x16x16_bf16: lane l = (q, j) supplies A[j][4q + t] and
// B[4q + t][j] for t = 0..3 as two packed bf16 pairs -- exactly the 4 k-steps the fp32 form
// takes from that lane (same permuted k), so one instruction replaces a 4-step fp32 chain and
// every fragment layout of the fp32 kernels is unchanged.  Operands are rounded to nearest-even
// (v_cvt_pk_bf16_f32); products are exact in fp32 and accumulate in fp32.
typedef float rs_f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// two fp32 -> one packed bf16 pair, carried in a float VGPR (lo in bits 0..15)
__device__ __forceinline__ float pack_bf16(float lo, float hi) {
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(float, v);
}

__device__ __forceinline__ rs_f32x4 mfma_bf16(float a01, float a23, float b01, float b23,
                                              rs_f32x4 c) {
  const s16x4 av = __builtin_bit_cast(s16x4, f32x2{a01, a23});
  const s16x4 bv = __builtin_bit_cast(s16x4, f32x2{b01, b23});
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(av, bv, c, 0, 0, 0);
}

// Wave-local LDS hand-off: make every lane's earlier LDS writes visible to the other lanes of the
// SAME wave and stop the compiler from moving LDS accesses across this point.  (DS instructions of
// one wave execute in order; the fences emit the lgkmcnt wait and pin the program order.)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS-only workgroup barrier: makes every wave's earlier LDS writes visible to the block and
// waits only for the wave's own LDS traffic (lgkmcnt).  __syncthreads()'s fence also drains vmcnt,
// i.e. it stalls each wave at every phase boundary until its outstanding global loads, stores and
// atomics (prefetches, a fused push) have completed.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// wait for this wave's outstanding vector-memory operations (global loads incl. the async
// global->LDS copies below, stores, atomics); follow with lds_barrier() to publish LDS-DMA data
__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Asynchronous copy of n4 float4 from global `src` to LDS `dst` by the whole block
// (global_load_lds_dwordx4: no VGPR round trip; each wave instruction writes 64 consecutive
// 16-B slots from the wave-uniform base in M0).  Complete after vm_wait_all() + lds_barrier().
// Issued from inline asm ON PURPOSE: through __builtin_amdgcn_global_load_lds the compiler
// cannot tell the DMA's LDS bytes from the kernel's other LDS data (one dynamic array) and puts
// an s_waitcnt vmcnt(0) in front of the next LDS read -- the prefetch would complete
// synchronously.  The compiler does not see these loads at all, so every vmcnt wait it emits
// for its own global loads is still correct (in-order return: it may only wait longer).
// The 32-bit LDS offset of a generic pointer into LDS, wave-uniform (readfirstlane).  The value
// goes through an empty asm first: otherwise the compiler folds the truncation past the
// readfirstlane into a 64-bit flat-pointer readfirstlane whose aperture half (src_shared_base)
// the gfx950 backend rejects ("Operand has incorrect register class") when the pointer is a
// loop-carried LDS buffer swap.
__device__ __forceinline__ uint32_t lds_addr_u32(const void* p) {
  uint32_t v = (uint32_t)(uintptr_t)p;
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ void glds_copy(float* dst, const float* src, int n4) {
  for (int k = threadIdx.x; k < n4; k += blockDim.x) {
    const int wbase = k - (int)(threadIdx.x & 63);  // wave-uniform
    const uint32_t lds = lds_addr_u32(dst + 4 * wbase);  // generic -> LDS offset
    const float* g = src + 4 * k;
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
}

// glds_copy for one wave (lanes 0..63 of the calling wave copy n4 float4; the other waves of the
// block are not involved).  Complete after vm_wait_all() + wave_lds_sync().
__device__ __forceinline__ void glds_copy_wave(float* dst, const float* src, int n4) {
  const int lane = (int)(threadIdx.x & 63);
  for (int k = lane; k < n4; k += 64) {
    const uint32_t lds = lds_addr_u32(dst + 4 * (k - lane));  // wave-uniform LDS base of this slot
    const float* g = src + 4 * k;
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
}

// glds_copy_wave for n 4-byte words (global_load_lds_dword: 64 words per wave instruction, any
// 4-B alignment).  Complete after vm_wait_all() + wave_lds_sync().
__device__ __forceinline__ void glds_copy_wave_u32(void* dst, const void* src, int n) {
  const int lane = (int)(threadIdx.x & 63);
  for (int k = lane; k < n; k += 64) {
    const uint32_t lds = lds_addr_u32(static_cast<uint32_t*>(dst) + (k - lane));
    const uint32_t* g = static_cast<const uint32_t*>(src) + k;
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
}

// Global dword load the compiler does not track (no vmcnt wait of its own): the caller waits with
// an explicit s_waitcnt naming the value (vm_wait_regs) before any use.
__device__ __forceinline__ float gload_untracked(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// The lane index through an empty volatile asm: every use re-derives it, so the compiler cannot
// hoist the dozens of lane-dependent LDS addresses of a fused kernel out of its sample loop and
// keep them live across every phase (measured on the InteractingLayer kernels: backward v2 167 ->
// 115 VGPRs, backward v3 from 400 B of scratch spills to 80, forward 52 -> 28 B).
__device__ __forceinline__ int lane_id() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t & 63;
}
// readfirstlane: the wave index is uniform, and saying so lets `if (wave_id() == k)` compile to a
// scalar branch instead of exec-mask save/restore around every guarded instruction
__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

// Sum over aligned groups of `W` lanes (W power of two, <= 64), result in every lane of the group.
// W <= 16 uses DPP row operations only (VALU, no LDS round trip): quad_perm xor-1 / xor-2, then
// row_half_mirror (lane i <-> 7 - i in each 8) and row_mirror (i <-> 15 - i in each 16): after
// each step every lane holds the sum of a symmetric group, so mirrors complete the butterfly.
// Wider groups finish with __shfl_xor (ds_bpermute / swizzle).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

template <int W>
__device__ __forceinline__ float group_sum(float v) {
  if (W >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  if (W >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  if (W >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror
  if (W >= 16) v += dpp_mov<0x140>(v); // row_mirror
#pragma unroll
  for (int o = 16; o < W; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------------------------
// Fill n 32-bit words with `value` as a kernel node.  Used instead of hipMemsetAsync on every
// path that callers capture into HIP graphs: a captured memset becomes a runtime-managed memset
// node, and the data-parallel AutoInt pool (several captured graphs replayed back to back)
// faulted only while such nodes were in its graphs.
// ---------------------------------------------------------------------------------------------
namespace {  // one copy per translation unit
__global__ void __launch_bounds__(256) rs_fill_u32_kernel(uint32_t* __restrict__ p, uint32_t value,
                                                         int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = value;
}

static inline void rs_fill_u32(hipStream_t s, void* p, uint32_t value, int64_t n) {
  if (n <= 0) return;
  int64_t grid = (n + 255) / 256;
  if (grid > 1024) grid = 1024;
  rs_fill_u32_kernel<<<(unsigned)grid, 256, 0, s>>>(reinterpret_cast<uint32_t*>(p), value, n);
}
}  // namespace

// ---------------------------------------------------------------------------------------------
// Counter-based dropout mask (shared bit-for-bit with oracle/ctr_oracle.py::dropout_keep).
// TF's stateful RNG cannot be reproduced, so the framework pins its own.  For the 64-bit layer
// seed s (splitmix64(seed + iteration)) and sample b, a per-sample key
//   kb = fmix32(lo32(s) ^ fmix32(hi32(s) + b))
// then per PAIR of keys (j, j ^ 1) one draw r = fmix32(kb ^ (h << 24 | i << 12 | (j & ~1)))
// (h < 256, i, j < 4096) whose 16-bit halves decide the two keys: keep iff
// half_j / 2^16 >= rate with half_j = j even ? r & 0xFFFF : r >> 16 (round 5; until then one
// 24-bit draw per element -- the per-score hash was a third of the many-field forward).
// fmix32 is the murmur3 finaliser: two 32-bit multiplies per draw (a 64-bit SplitMix costs ~3x
// more on the VALU), and kb is hoisted per sample.  A 2^-16 probability granularity: rate 0.2
// keeps 0.799988 of the scores instead of 0.8.
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint32_t dropout_sample_key(uint64_t seed, uint32_t b) {
  return fmix32((uint32_t)seed ^ fmix32((uint32_t)(seed >> 32) + b));
}

__device__ __forceinline__ uint32_t dropout_half(uint32_t r, uint32_t j) {
  return (j & 1u) ? (r >> 16) : (r & 0xFFFFu);
}
__device__ __forceinline__ bool dropout_keep_k(uint32_t kb, uint32_t h, uint32_t i, uint32_t j,
                                               float rate) {
  const uint32_t r = fmix32(kb ^ ((h << 24) | (i << 12) | (j & ~1u)));
  return (float)dropout_half(r, j) * (1.0f / 65536.0f) >= rate;
}

// the same decision against an integer threshold (dropout_thr16(rate) = ceil(rate * 2^16)):
// half * 2^-16 >= rate  <=>  half >= ceil(rate * 2^16), both sides exact -- bit-identical masks
// without the convert / multiply; a kernel sweeping keys in order draws once per key pair
// (dropout_draw) and tests both halves
__host__ __device__ __forceinline__ uint32_t dropout_thr16(float rate) {
  return (uint32_t)ceilf(rate * 65536.0f);
}
__device__ __forceinline__ uint32_t dropout_draw(uint32_t kb, uint32_t h, uint32_t i, uint32_t j) {
  return fmix32(kb ^ ((h << 24) | (i << 12) | (j & ~1u)));
}

__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint32_t b, uint32_t h, uint32_t i,
                                             uint32_t j, float rate) {
  return dropout_keep_k(dropout_sample_key(seed, b), h, i, j, rate);
}

// ---------------------------------------------------------------------------------------------
// Deterministic column reduction of per-block partial rows:
//   out[c] (+)= sum_r part[r * ld + c]   (c < ncols; columns >= split go to out1[c - split])
// Block = 64 columns x G row-groups; each thread sums rows r = g, g+G, ... in order, then the G
// partial sums are combined in g order: a fixed summation order for a given (nrows, G), so the
// result is bitwise reproducible.  Many columns per wave keep the loads coalesced; the G row
// groups keep G independent load streams per column in flight.
// ---------------------------------------------------------------------------------------------
template <int G>
__global__ void __launch_bounds__(64 * G) column_reduce_kernel(
    const float* __restrict__ part, int nrows, int64_t ld, int64_t ncols, int64_t split,
    float* __restrict__ out0, float* __restrict__ out1, int accumulate) {
  __shared__ float red[G][64];
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lc;
  float s = 0.f;
  if (c < ncols) {
#pragma unroll 4
    for (int r = g; r < nrows; r += G) s += part[(int64_t)r * ld + c];
  }
  red[g][lc] = s;
  __syncthreads();
  if (g == 0 && c < ncols) {
    float t = red[0][lc];
#pragma unroll
    for (int k = 1; k < G; ++k) t += red[k][lc];
    float* d = c < split ? out0 + c : out1 + (c - split);
    *d = accumulate ? (*d + t) : t;
  }
}

static inline void launch_column_reduce(hipStream_t s, const float* part, int nrows, int64_t ld,
                                        int64_t ncols, int64_t split, float* out0, float* out1,
                                        int accumulate) {
  const unsigned grid = (unsigned)((ncols + 63) / 64);
  column_reduce_kernel<16><<<grid, 64 * 16, 0, s>>>(part, nrows, ld, ncols, split, out0, out1,
                                                    accumulate);
}

// ---------------------------------------------------------------------------------------------
// "The last workgroup of this launch" without a second launch: a completion counter sharded over
// 8 sub-counters (blockIdx % 8, one 128-B line each) plus a top counter, so at most
// ceil(grid / 8) + 8 arrivals meet on any one word (one device-scope atomic serialises ~12 ns at
// the memory side; 1024 arrivals on one word would cost ~13 us).  The counters live in
// caller-owned memory, int32[RS_DONE_WORDS], all zero between launches: each sub-counter is reset
// by its own last arriver and the top counter by the global last arriver (atomic exchanges, the
// same memory-side path as the adds).  Every thread of the block must call this; it returns true
// in thread 0 of the last block only.  No memory fence: callers use it only to order their own
// earlier LOADS (consumed values) before a reset done by the last block.
// ---------------------------------------------------------------------------------------------
// id -> table row (embedding.hip header): row = base + H(id) mod bucket, H = identity or SplitMix64
// ---------------------------------------------------------------------------------------------
enum { RS_HASH_MOD = 0, RS_HASH_SPLITMIX = 1 };

__device__ __forceinline__ int64_t hash_row(int64_t id, int64_t base, int64_t bucket, int mode) {
  uint64_t u = (uint64_t)id;
  if (mode == RS_HASH_SPLITMIX) u = splitmix64(u);
  // same value either way; a 64-bit remainder is a long emulated sequence on the GPU, the 32-bit
  // one a few VALU ops (Criteo-style ids and per-field buckets fit in 32 bits)
  if (((u | (uint64_t)bucket) >> 32) == 0) return base + (int64_t)((uint32_t)u % (uint32_t)bucket);
  return base + (int64_t)(u % (uint64_t)bucket);
}

// ---------------------------------------------------------------------------------------------
#define RS_DONE_STRIDE 32
#define RS_DONE_WORDS (9 * RS_DONE_STRIDE)
// nblocks: the blocks taking part (blocks 0 .. nblocks - 1; default the whole grid)
// nblocks / bid: the blocks taking part and this block's index among them (default: the whole
// grid, blockIdx.x)
__device__ __forceinline__ bool rs_last_block(int32_t* ctr, int nblocks = -1, int bid = -1) {
  __syncthreads();
  if (threadIdx.x != 0) return false;
  const unsigned G = nblocks < 0 ? gridDim.x : (unsigned)nblocks;
  const unsigned k = (bid < 0 ? blockIdx.x : (unsigned)bid) & 7u;
  const int nk = (int)((G - k + 7u) / 8u);
  const int nsub = (int)(G < 8u ? G : 8u);
  int32_t* sub = ctr + k * RS_DONE_STRIDE;
  int32_t* top = ctr + 8 * RS_DONE_STRIDE;
  if (atomicAdd(sub, 1) != nk - 1) return false;
  atomicExch(sub, 0);
  if (atomicAdd(top, 1) != nsub - 1) return false;
  atomicExch(top, 0);
  return true;
}

// ---------------------------------------------------------------------------------------------
// Scan-mode row mark: flag[row] = -2 with a plain store (idempotent: the hot rows of a Zipf
// batch receive thousands of marks, which coalesce in L2; an atomic bitmap update serialised
// them at the memory side and cost the InteractingLayer backward ~10 us).  Clean state is -1,
// shared with list mode.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void scan_mark(int32_t* flag, int64_t row) { flag[row] = -2; }
