// Shared device helpers for the Light-3D-U-Net gfx950 kernels.
// Layout convention: every activation is NCDHW fp32 with the spatial volume
// S = D*H*W contiguous per (n, c); a tensor view is (base pointer, batch stride in elements).
// Channel stride is always S.  A batch stride larger than C*S lets a kernel read/write one
// channel range of a concatenation buffer in place (zero-copy torch.cat, unet3d.py:141).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "l3u.h"

#define L3U_DEV __device__ __forceinline__
#define L3U_INLINE_HOST static inline

namespace l3u {

constexpr float kSlope = 0.01f;   // LeakyReLU(0.01)   unet3d.py:52,63
constexpr float kEps = 1e-5f;     // InstanceNorm3d eps (torch default)  unet3d.py:51

// Per-(n,c) InstanceNorm record written by in_finalize and read by every consumer.
//  [0] mean  [1] rstd  [2] scale = k*gamma*rstd  [3] shift = k*beta
//  [4] k (Dropout3d keep scale: 0 or 1/(1-p); 1 when no dropout)  [5] gamma  [6] beta
//  [7] rank-1 scale of the normalised operand (l3u_norm_src.rank1[c]; 0: a full tensor)
// With the dropout scale folded in, the forward transform is  a = lrelu(scale*(y - mean) + shift),
// valid because lrelu(k*v) = k*lrelu(v) for k >= 0.  (y - mean) is formed first: folding the mean
// into the shift cancels catastrophically when |mean| >> std and costs ~1e-5 relative accuracy.
constexpr int kRec = 8;

// ---- activation storage types -----------------------------------------------------------------
// Activations (and their gradients) are stored as T = float or bf16; every kernel computes in fp32
// (loads widen, stores round to nearest even with v_cvt_pk_bf16_f32), statistics in fp32 / fp64,
// weights and partial sums stay fp32.  Overloads on the pointer type, so the same kernel text
// serves LDS (float) and global (T) operands.
typedef __bf16 bf16;
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef float f2_t __attribute__((ext_vector_type(2)));
typedef __bf16 b4_t __attribute__((ext_vector_type(4)));
typedef __bf16 b2_t __attribute__((ext_vector_type(2)));

L3U_DEV f4_t ldv4(const float* p) { return *reinterpret_cast<const f4_t*>(p); }
L3U_DEV f4_t ldv4(const bf16* p) { return __builtin_convertvector(*reinterpret_cast<const b4_t*>(p), f4_t); }
// L3U_ST_NT=1: the generic tensor stores below non-temporal (streamed past the XCD's L2, which the
// next launch cannot hit anyway: the kernel-boundary release writes it back, the acquire
// invalidates it)
#ifndef L3U_ST_NT
#define L3U_ST_NT 0
#endif
template <typename V>
L3U_DEV void st_pol(V* p, V v) {
  if constexpr (L3U_ST_NT != 0) __builtin_nontemporal_store(v, p); else *p = v;
}
L3U_DEV void stv4(float* p, f4_t v) { st_pol(reinterpret_cast<f4_t*>(p), v); }
L3U_DEV void stv4(bf16* p, f4_t v) { st_pol(reinterpret_cast<b4_t*>(p), __builtin_convertvector(v, b4_t)); }
L3U_DEV void stv4_nt(float* p, f4_t v) { __builtin_nontemporal_store(v, reinterpret_cast<f4_t*>(p)); }
L3U_DEV void stv4_nt(bf16* p, f4_t v) {
  __builtin_nontemporal_store(__builtin_convertvector(v, b4_t), reinterpret_cast<b4_t*>(p));
}
L3U_DEV f2_t ldv2(const float* p) { return *reinterpret_cast<const f2_t*>(p); }
L3U_DEV f2_t ldv2(const bf16* p) { return __builtin_convertvector(*reinterpret_cast<const b2_t*>(p), f2_t); }
L3U_DEV void stv2(float* p, f2_t v) { st_pol(reinterpret_cast<f2_t*>(p), v); }
L3U_DEV void stv2(bf16* p, f2_t v) { st_pol(reinterpret_cast<b2_t*>(p), __builtin_convertvector(v, b2_t)); }
// v rounded to the storage precision of T (the value a store + reload would give)
L3U_DEV f4_t round_to(f4_t v, const float*) { return v; }
L3U_DEV f4_t round_to(f4_t v, const bf16*) { return __builtin_convertvector(__builtin_convertvector(v, b4_t), f4_t); }
L3U_DEV float ld1(const float* p) { return *p; }
L3U_DEV float ld1(const bf16* p) { return (float)*p; }
L3U_DEV void st1(float* p, float v) { st_pol(p, v); }
L3U_DEV void st1(bf16* p, float v) { st_pol(p, (bf16)v); }

// a * b rounded on its own, never contracted into a following add (an FMA would round once and
// differ from the product that was stored: the rank-1 operands must equal the materialised tensor)
// (__fmul_rn is a plain contractible multiply on this toolchain: the empty asm fences the product)
L3U_DEV float mul_rn(float a, float b) {
  float p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}
L3U_DEV f4_t mul_rn(f4_t v, float s) {
  f4_t p = v * s;
  asm volatile("" : "+v"(p));
  return p;
}

L3U_DEV float lrelu(float v) { return v > 0.f ? v : v * kSlope; }
L3U_DEV float lrelu_d(float pre) { return pre > 0.f ? 1.f : kSlope; }   // torch: x > 0 ? 1 : slope

// Wave-wide sums without LDS traffic: DPP butterflies inside each 16-lane row (quad_perm xor 1,
// xor 2, half-mirror, mirror), then the gfx950 permlane16/32 swaps across rows.  Every lane ends
// with the same value, summed in the same order (a+b == b+a), so the result is deterministic.
template <int CTRL>
L3U_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
L3U_DEV float swap_sum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
L3U_DEV float swap_sum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
L3U_DEV float row_sum16(float v) {   // sum over the 16 lanes of a DPP row, in every lane
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror
  return v;
}
L3U_DEV float wave_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror
  return swap_sum32(swap_sum16(v));
}

// Block-wide sum for 256-thread blocks; every thread gets the result.  `red` >= 4 floats of LDS.
L3U_DEV float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

template <int CTRL>
L3U_DEV double dpp_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffffu), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// fp64 sum over the 16 lanes of a DPP row (fixed order: deterministic), in every lane
L3U_DEV double row_sum16d(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return v;
}
L3U_DEV double swap_sum_d(double v, bool row16) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)(u & 0xffffffffu), hi = (unsigned)(u >> 32);
  const auto rl = row16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto rh = row16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const double a = __longlong_as_double((long long)(((unsigned long long)rh[0] << 32) | rl[0]));
  const double b = __longlong_as_double((long long)(((unsigned long long)rh[1] << 32) | rl[1]));
  return a + b;
}
L3U_DEV double wave_sum_d(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return swap_sum_d(swap_sum_d(v, true), false);
}

// Block-wide fp64 sum for 256-thread blocks (cross-block gradient sums of InstanceNorm backward
// are cancellation-heavy: they are accumulated and stored in fp64).  `red` >= 4 doubles of LDS.
L3U_DEV double block_sum256d(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// t[v] = sum_{i < n} p[i * NV + v] in index order (fp64); the loads of 8 steps are issued
// together so a long partial list costs one memory latency per 8 entries, not one per entry.
template <int NV>
L3U_DEV void seq_sum(const double* __restrict__ p, int n, double t[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v) t[v] = 0.0;
  for (int i0 = 0; i0 < n; i0 += 8) {
    // clamped unconditional loads (a predicated load became a branch with a vmcnt(0) behind it)
    double a[8][NV];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < NV; ++v) a[u][v] = p[min(i0 + u, n - 1) * NV + v];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + u < n) {
#pragma unroll
        for (int v = 0; v < NV; ++v) t[v] += a[u][v];
      }
  }
}

L3U_DEV unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// A load from a workgroup-uniform address issued as a VECTOR load (global_load, counted by
// vmcnt, in order).  A uniform load would otherwise be a scalar load (s_load), and scalar loads
// complete out of order: every later use of ANY scalar load -- a kernel argument fetched lazily
// inside a branch included -- then waits with lgkmcnt(0) for all of them.  In the small-level
// IN consumers that chained the record's inputs (gamma / beta, then the Dropout3d step and rank-1
// scale, then the kernel-argument base of the partials) into three extra memory round trips
// before the partials were even requested (round 6 wave stamps, dwv_fwd at 6^3: partials in
// registers 3.5 us after the wave began, the data 1.5 us).  The opaque zero (a VGPR the compiler
// cannot prove uniform) makes the address per-lane.
template <typename V>
L3U_DEV V vld(const V* p) {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return p[z];
}

// Kernel arguments all requested at the kernel's entry, in one batch of scalar loads with one
// wait.  Left alone, hipcc loads each argument where it is first used: behind a uniform branch (a
// paired launch's second problem, an optional operand) that is a scalar-load round trip, then a
// wait, then the next batch -- up to four dependent round trips before the first vector load of
// the pointwise GEMMs (ISA: s_load ... s_waitcnt lgkmcnt(0) pairs ahead of the first
// global_load).  An empty asm that takes every argument in SGPRs makes them all live at entry.
// Measured per kernel family (A/B): kept for the pointwise forwards (-3 us/step) and
// the block tails (-2.5 us); the pointwise backwards, out_conv / front / reduction launches and
// the ConvTranspose3d backward got slower or stayed equal (higher register counts), and the
// stencil kernels spilled.
template <typename A>
L3U_DEV void karg_pin(const A& a) { asm volatile("" ::"s"(a)); }
template <typename... A>
L3U_DEV void kargs_now(const A&... a) { (karg_pin(a), ...); }

// the record's per-channel inputs (affine parameters, Dropout3d step, rank-1 scale), vector
// loads issued with the partials so that all of them arrive in one memory round trip
struct RecIn { float g, b, rk1; int st; };
L3U_DEV RecIn record_inputs(const l3u_norm_src& s, int c) {
  RecIn q;
  q.g = s.gamma ? vld(s.gamma + c) : 1.f;
  q.b = s.beta ? vld(s.beta + c) : 0.f;
  q.st = (s.drop_p > 0.f && s.step) ? vld(s.step) : 0;
  q.rk1 = s.rank1 ? vld(s.rank1 + c) : 0.f;
  return q;
}
L3U_DEV void record_from(const l3u_norm_src& s, const RecIn& q, int n, int c, int C, float cn,
                         float mu, float m2, float r[kRec]);

// Merge the (count, mean, M2) partials of one (n, c) with the 64 lanes of the calling wave and
// build the 8-float record.  Two passes of plain wave sums (DPP, no LDS): the total count and
// sum of count * mean give the mean; then every partial's M2 plus count * (mean_i - mean)^2 --
// all non-negative terms -- sum to the M2 of the whole (n, c).  Fixed order: every caller for
// the same (n, c) gets bit-identical values.  (Round 4 merged pairs with Chan's formula along a
// 6-round shuffle tree: ~3.5 us on the critical path of every IN-consuming small-level launch,
// wave stamps r5d.)  Must be called by a full wave; returns the record in `r` on every lane.
//
// Split in two so that a consumer can request the partials FIRST, before its data loads, and
// finish the record after issuing them (record_pre / record_finish): up to 512 partials are 8
// clamped unconditional loads per lane in straight-line code (a loop, or a branch around each
// load, makes hipcc wait for every outstanding load -- vmcnt(0) -- before requesting them).
struct RecPre {
  float v[8][3];
  RecIn q;
};
// raw loads only (the masking happens at the first use, in record_finish: a select right here
// would make hipcc wait for the loads before the caller's next requests)
L3U_DEV void rec_fetch8(const float* p, int nsb, int i0, float (&v)[8][3]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int ic = min(i0 + 64 * u, nsb - 1);
    v[u][0] = p[ic * 3];
    v[u][1] = p[ic * 3 + 1];
    v[u][2] = p[ic * 3 + 2];
  }
}
L3U_DEV void rec_mask8(int nsb, int i0, float (&v)[8][3]) {   // zero the entries past the list
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const bool ok = i0 + 64 * u < nsb;
    v[u][0] = ok ? v[u][0] : 0.f;
    v[u][1] = ok ? v[u][1] : 0.f;
    v[u][2] = ok ? v[u][2] : 0.f;
  }
}
L3U_DEV void record_pre(const l3u_norm_src& s, int n, int c, int C, RecPre& rp) {
  rp.q = record_inputs(s, c);
  const float* p = s.stat_part + ((long long)n * C + c) * s.nsb * 3;
  if (s.nsb <= 512) rec_fetch8(p, s.nsb, threadIdx.x & 63, rp.v);
}
L3U_DEV void record_finish(const l3u_norm_src& s, RecPre& rp, int n, int c, int C, float r[kRec]) {
  const int l = threadIdx.x & 63;
  const float* p = s.stat_part + ((long long)n * C + c) * s.nsb * 3;
  float (&v)[8][3] = rp.v;
  float cs = 0.f, ms = 0.f;
  if (s.nsb <= 512) {
    rec_mask8(s.nsb, l, v);
#pragma unroll
    for (int u = 0; u < 8; ++u) { cs += v[u][0]; ms = fmaf(v[u][0], v[u][1], ms); }
  } else {   // long lists (config 5's 64^3 GEMMs: 1024 partials): re-read in the second pass
    for (int i0 = l; i0 < s.nsb; i0 += 512) {
      rec_fetch8(p, s.nsb, i0, v);
      rec_mask8(s.nsb, i0, v);
#pragma unroll
      for (int u = 0; u < 8; ++u) { cs += v[u][0]; ms = fmaf(v[u][0], v[u][1], ms); }
    }
  }
  const float cn = wave_sum(cs);
  const float mu = cn > 0.f ? wave_sum(ms) / cn : 0.f;
  float m2 = 0.f;
  auto add_m2 = [&] {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float d = v[u][1] - mu;
      m2 += fmaf(v[u][0] * d, d, v[u][2]);
    }
  };
  if (s.nsb <= 512) {
    add_m2();   // the lane's partials are still in registers (zeros where it holds none)
  } else {
    for (int i0 = l; i0 < s.nsb; i0 += 512) {
      rec_fetch8(p, s.nsb, i0, v);
      rec_mask8(s.nsb, i0, v);
      add_m2();
    }
  }
  record_from(s, rp.q, n, c, C, cn, mu, wave_sum(m2), r);
}
L3U_DEV void finalize_record(const l3u_norm_src& s, int n, int c, int C, float r[kRec]) {
  RecPre rp;
  record_pre(s, n, c, C, rp);
  record_finish(s, rp, n, c, C, r);
}

// The record of (n, c) from its merged (count, mean, M2): rstd, the affine parameters and the
// Dropout3d keep scale of (step, layer, n*C + c).
L3U_DEV void record_from(const l3u_norm_src& s, const RecIn& q, int n, int c, int C, float cn,
                         float mu, float m2, float r[kRec]) {
  const float var = cn > 0.f ? m2 / cn : 0.f;
  const float rstd = 1.0f / sqrtf(var + kEps);
  const float g = q.g, b = q.b;
  float k = 1.f;
  if (s.drop_p > 0.f) {
    const int st = q.st;
    const unsigned long long h = splitmix64(s.seed ^ splitmix64(((unsigned long long)st << 32) ^
                                                                ((unsigned long long)s.layer << 24) ^
                                                                (unsigned long long)(n * C + c)));
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
    k = u < s.drop_p ? 0.f : 1.f / (1.f - s.drop_p);
  }
  r[0] = mu;
  r[1] = rstd;
  r[2] = k * g * rstd;
  r[3] = k * b;
  r[4] = k;
  r[5] = g;
  r[6] = b;
  r[7] = q.rk1;
}

// Workgroup-level: wave 0 finalizes, broadcasts through `sh8` (8 floats of LDS) and, if asked,
// stores the record for the backward.  All threads must call it (contains a barrier).
L3U_DEV void block_record(const l3u_norm_src& s, int n, int c, int C, bool store, float* sh8) {
  if (threadIdx.x < 64) {
    float r[kRec];
    finalize_record(s, n, c, C, r);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int i = 0; i < kRec; ++i) sh8[i] = r[i];
      if (store && s.rec_out) {
        float* o = s.rec_out + ((long long)n * C + c) * kRec;
#pragma unroll
        for (int i = 0; i < kRec; ++i) o[i] = r[i];
      }
    }
  }
  __syncthreads();
}

// Two records at once (waves 0 and 1 merge in parallel), one barrier; sh8: 16 floats of LDS.
// field-wise selects: a reference picked at run time between the two by-value kernel arguments
// made the compiler copy both to scratch in every thread (120 B of private memory per thread,
// ~25 MB of HBM writes per 48^3 launch, profiles/r1i_pmc_step.json)
L3U_DEV l3u_norm_src pick_src(const l3u_norm_src& a, const l3u_norm_src& b, bool q) {
  l3u_norm_src s;
  s.stat_part = q ? a.stat_part : b.stat_part;
  s.nsb = q ? a.nsb : b.nsb;
  s.layer = q ? a.layer : b.layer;
  s.gamma = q ? a.gamma : b.gamma;
  s.beta = q ? a.beta : b.beta;
  s.drop_p = q ? a.drop_p : b.drop_p;
  s.seed = q ? a.seed : b.seed;
  s.step = q ? a.step : b.step;
  s.rec_out = q ? a.rec_out : b.rec_out;
  s.rank1 = q ? a.rank1 : b.rank1;
  return s;
}
// split form: the merging waves request the records' loads (block_record2_pre) BEFORE the
// caller's streamed loads -- vector loads complete in order, so records requested behind the
// data could only be merged once the data had arrived -- and merge them after (block_record2_fin)
L3U_DEV void block_record2_pre(const l3u_norm_src& a, const l3u_norm_src& b, bool has_b, int n,
                               int c, int C, RecPre& rp) {
  const int wv = threadIdx.x >> 6;
  if (wv == 0 || (wv == 1 && has_b)) record_pre(pick_src(a, b, wv == 0), n, c, C, rp);
}
L3U_DEV void block_record2_fin(const l3u_norm_src& a, const l3u_norm_src& b, bool has_b, int n,
                               int c, int C, bool store, float* sh8, RecPre& rp) {
  const int wv = threadIdx.x >> 6;
  if (wv == 0 || (wv == 1 && has_b)) {
    const l3u_norm_src s = pick_src(a, b, wv == 0);
    float r[kRec];
    record_finish(s, rp, n, c, C, r);
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
      for (int i = 0; i < kRec; ++i) sh8[wv * 8 + i] = r[i];
      if (store && s.rec_out) {
        float* o = s.rec_out + ((long long)n * C + c) * kRec;
#pragma unroll
        for (int i = 0; i < kRec; ++i) o[i] = r[i];
      }
    }
  }
  __syncthreads();
}
L3U_DEV void block_record2(const l3u_norm_src& a, const l3u_norm_src& b, bool has_b, int n, int c,
                           int C, bool store, float* sh8) {
  RecPre rp;
  block_record2_pre(a, b, has_b, n, c, C, rp);
  block_record2_fin(a, b, has_b, n, c, C, store, sh8, rp);
}

// a / b for 0 <= a < 2^24, b > 0, with inv = 1.f / b: one float multiply and a correction step
// (the float quotient is within 1 of the exact one) instead of an integer division
L3U_DEV int fdiv(int a, int b, float inv) {
  int q = (int)((float)a * inv);
  const int r = a - q * b;
  q += r < 0 ? -1 : (r >= b ? 1 : 0);
  return q;
}

// MaxPool3d(2, 2) backward folded into a consumer's load (DownBlock, unet3d.py:104): the gradient
// of the pooled level's input at the x-quad (z, y, x..x+3) (x % 4 == 0, even D / H, W % 4 == 0)
// is v (the skip-connection gradient quad) plus dpool of the window's argmax (idx = 4dz + 2dy + dx
// per pooled voxel, l3u_maxpool2_fwd's encoding) -- l3u_maxpool2_bwd's expression, bit for bit.
// dpp / ipp: the (n, c) planes of dpool [Ho*Wo*Do] and idx; H, W: the fine level's plane.
// Split form for kernels that request every operand before the first use: unpool_tap loads the
// pooled gradient pair and its argmax code, unpool_apply adds them (same expression).
struct UnpoolTap { f2_t g; int id; };
L3U_DEV UnpoolTap unpool_tap(const float* __restrict__ dpp, const unsigned char* __restrict__ ipp,
                             int z, int y, int x, int H, int W) {
  const long long o2 = ((long long)(z >> 1) * (H >> 1) + (y >> 1)) * (W >> 1) + (x >> 1);
  return {*reinterpret_cast<const f2_t*>(dpp + o2), reinterpret_cast<const unsigned short*>(ipp)[o2 >> 1]};
}
L3U_DEV f4_t unpool_apply(f4_t v, UnpoolTap t, int z, int y) {
  const int i0 = t.id & 0xff, i1 = t.id >> 8, j = 2 * (z & 1) + (y & 1);
  v[0] += i0 == 2 * j ? t.g.x : 0.f;
  v[1] += i0 == 2 * j + 1 ? t.g.x : 0.f;
  v[2] += i1 == 2 * j ? t.g.y : 0.f;
  v[3] += i1 == 2 * j + 1 ? t.g.y : 0.f;
  return v;
}
L3U_DEV f4_t unpool_add(f4_t v, const float* __restrict__ dpp, const unsigned char* __restrict__ ipp,
                        int z, int y, int x, int H, int W) {
  return unpool_apply(v, unpool_tap(dpp, ipp, z, y, x, H, W), z, y);
}

// XCD-aware block remap (guide §5.5 T1, bijective form): blocks that share halo planes / weight
// tiles are consecutive in the logical order, and consecutive logical ids land on one XCD.
L3U_DEV int xcd_remap(int bid, int nblocks) {
  if (nblocks < 16) return bid;
  const int xcd = bid & 7, q = nblocks >> 3, r = nblocks & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Wave stamps (profiling variant builds only, -DL3U_STAMP; tools/stamp.py): lane 0 of every wave
// of a launch with at most kStampMaxWaves waves records {begin, end} in wall-clock ticks (100 MHz),
// the kernel id (L3U_STAMP_SCOPE in each kernel) and the flat block index into a device buffer
// that l3u_stamp_setup installs (256 shards of cap / 256 records, one counter each).  Product builds compile the scope to nothing.
#ifdef L3U_STAMP
struct StampRec { unsigned long long t0, t1, m0, m1; unsigned id, blk, nwg, pad, r0, r1; };
constexpr unsigned kStampMaxWaves = 65536;
static __device__ StampRec* l3u_stamp_dptr;
static __device__ unsigned* l3u_stamp_dctr;
static __device__ unsigned l3u_stamp_cap;
void stamp_register(void (*set)(void*, void*, unsigned));
static void l3u_stamp_set_tu(void* b, void* c, unsigned cap) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(l3u_stamp_dptr), &b, sizeof b);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(l3u_stamp_dctr), &c, sizeof c);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(l3u_stamp_cap), &cap, sizeof cap);
}
static const int l3u_stamp_reg = (stamp_register(l3u_stamp_set_tu), 0);
struct StampScope {   // the slot is taken at wave begin (the atomic's return overlaps the body)
  unsigned long long t0, m[2];
  unsigned id, slot, shard;
  bool on;
  __device__ void mark(int k) { m[k] = wall_clock64(); }   // intermediate stage stamps
  __device__ explicit StampScope(unsigned i) : m{0, 0}, id(i), slot(0), shard(0) {
    t0 = wall_clock64();
    const unsigned long long nwv = (blockDim.x * blockDim.y * blockDim.z + 63) / 64;
    on = l3u_stamp_dptr != nullptr && (threadIdx.x & 63) == 0 &&
         (unsigned long long)gridDim.x * gridDim.y * gridDim.z * nwv <= kStampMaxWaves;
    if (on) {   // 256 counters (by block): no fan-in on one word
      shard = (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) & 255;
      slot = atomicAdd(l3u_stamp_dctr + shard, 1u);
    }
  }
  __device__ ~StampScope() {
    if (on) {
      const unsigned long long t1 = wall_clock64();
      if (slot < l3u_stamp_cap / 256) {
        const unsigned blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        l3u_stamp_dptr[shard * (l3u_stamp_cap / 256) + slot] =
            StampRec{t0, t1, m[0], m[1], id, blk * 16 + threadIdx.x / 64,
                     gridDim.x * gridDim.y * gridDim.z, 1, 0, 0};
      }
    }
  }
};
#define L3U_STAMP_SCOPE(ID) l3u::StampScope l3u_stamp_scope_(ID)
#define L3U_STAMP_MARK(K) l3u_stamp_scope_.mark(K)
#else
#define L3U_STAMP_SCOPE(ID) ((void)0)
#define L3U_STAMP_MARK(K) ((void)0)
#endif

// ConvTranspose3d(k2, s2) backward tile kernel (convt.hip): weight/bias partial count (0: shape
// not taken) and the launch; same partial layout as l3u_convt_bwd_fused
int convt_tile_nparts(int N, int Ci, int Co, int D, int H, int W);
template <typename T>
int convt_tile_launch(const float* dy, long long dy_nstride, const T* x, long long x_nstride,
                      const float* w, float* dx, long long dx_nstride, float* wpart, float* bpart,
                      int N, int Ci, int Co, int D, int H, int W, hipStream_t stream);

}  // namespace l3u

// C-ABI twins: every activation entry point exists for fp32 and, with the suffix _bf16, for bf16
// storage (l3u_bf16 = the raw 16-bit pattern in the header).  bp() maps an ABI pointer to the
// kernel element type (identity for float), so both twins share one argument list.
L3U_INLINE_HOST const float* bp(const float* p) { return p; }
L3U_INLINE_HOST float* bp(float* p) { return p; }
L3U_INLINE_HOST const l3u::bf16* bp(const l3u_bf16* p) { return reinterpret_cast<const l3u::bf16*>(p); }
L3U_INLINE_HOST l3u::bf16* bp(l3u_bf16* p) { return reinterpret_cast<l3u::bf16*>(p); }
#define L3U_TWIN(NAME, PARAMS, ...)                               \
  extern "C" int NAME PARAMS(float) { return __VA_ARGS__; }        \
  extern "C" int NAME##_bf16 PARAMS(l3u_bf16) { return __VA_ARGS__; }

// Error plumbing for the C-ABI: every entry point returns a hipError_t as int.
#define L3U_CHECK_LAUNCH() return (int)hipGetLastError()
#define L3U_REQUIRE(cond) \
  do {                    \
    if (!(cond)) return (int)hipErrorInvalidValue; \
  } while (0)
