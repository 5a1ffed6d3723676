// InstanceNorm3d(affine) + LeakyReLU + Dropout3d + residual — statistics finalize, fused apply,
// and the two-phase backward.  Replaces nn.InstanceNorm3d / nn.LeakyReLU / nn.Dropout3d and the
// residual add of ResidualBlock.forward (unet3d.py:51-52, 62-66, 72, 77-93).
//
// Forward statistics come from the producing GEMM's epilogue as (count, mean, M2) partials per
// (n, c, voxel-block); in_finalize merges them (Chan, fixed tree order -> deterministic) into the
// per-(n,c) record of common.h.  All elementwise kernels are one workgroup per (n, c, voxel range)
// so the record is a workgroup-uniform scalar load, and loads/stores are float4 when aligned.
#include "common.h"
using namespace l3u;

typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

// one wave per (n, c)
__global__ __launch_bounds__(256) void in_finalize_kernel(l3u_norm_src src, int NC, int C) {
  L3U_STAMP_SCOPE(301);
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (wid >= NC) return;
  float r[kRec];
  finalize_record(src, wid / C, wid % C, C, r);
  if (l == 0) {
    float* o = src.rec_out + (long long)wid * kRec;
#pragma unroll
    for (int i = 0; i < kRec; ++i) o[i] = r[i];
  }
}

// out = lrelu(scale2*(y2-mean2) + shift2 + R),  R = r (identity) or scale_r*(r-mean_r) + shift_r.
// With HAS_SRC the records are finalized here from the GEMM partials (no in_finalize launch);
// workgroup x == 0 of each (n, c) stores them for the backward.
template <typename T, bool VEC, bool HAS_SRC, bool RK = false>
__global__ __launch_bounds__(256) void norm_act_fwd_kernel(
    const T* __restrict__ y2, long long y2ns, const float* __restrict__ rec2, l3u_norm_src src2,
    const T* __restrict__ r, long long rns, const float* __restrict__ recr, l3u_norm_src srcr,
    int shortcut, T* __restrict__ out, long long ons, int C, int S) {
  L3U_STAMP_SCOPE(302);
  kargs_now(y2, y2ns, rec2, r, rns, recr, shortcut, out, ons, C, S);
  __shared__ float sh[16];
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  // RK (rns < 0): rank-1 residual, record_r[7] * one stored channel (include/l3u.h)
  constexpr bool rk = RK;
  const T* yp = y2 + (long long)n * y2ns + (long long)c * S;
  const T* rp = r + (long long)n * (rk ? -rns : rns) + (rk ? 0ll : (long long)c * S);
  T* op = out + (long long)n * ons + (long long)c * S;
  // the records' partial sums are requested first, then the first tile (one round trip for both;
  // the merge waits only for the loads ahead of the tile); every later tile one iteration ahead
  const int i0 = (blockIdx.x * 256 + threadIdx.x) * 4, istep = gridDim.x * 1024;
  RecPre rpre;   // the records' loads before the tile's (common.h block_record2_pre)
  if (HAS_SRC) block_record2_pre(src2, srcr, shortcut != 0, n, c, C, rpre);
  // (requests clamped to the last tile instead of branched: a load behind a branch makes every
  // later wait assume the worst about what is in flight)
  f4 yv = {0.f, 0.f, 0.f, 0.f}, rv = yv;
  if (VEC) { const int ic = min(i0, S - 4); yv = ldv4(yp + ic); rv = ldv4(rp + ic); }
  float m2, a2, b2, ar = 1.f, br = 0.f, mr = 0.f, rks = 1.f;
  if (HAS_SRC) {
    block_record2_fin(src2, srcr, shortcut != 0, n, c, C, blockIdx.x == 0, sh, rpre);
    m2 = sh[0]; a2 = sh[2]; b2 = sh[3];
    if (shortcut) { mr = sh[8]; ar = sh[10]; br = sh[11]; rks = sh[15]; }
  } else {
    m2 = rec2[(long long)nc * kRec + 0];
    a2 = rec2[(long long)nc * kRec + 2];
    b2 = rec2[(long long)nc * kRec + 3];
    if (shortcut) {
      mr = recr[(long long)nc * kRec + 0];
      ar = recr[(long long)nc * kRec + 2];
      br = recr[(long long)nc * kRec + 3];
      rks = recr[(long long)nc * kRec + 7];
    }
  }
  if (VEC) {
    for (int i = i0; i < S; i += istep) {
      const int in_ = min(i + istep, S - 4);
      const f4 yn = ldv4(yp + in_), rn = ldv4(rp + in_);
      if (rk) rv = mul_rn(rv, rks);
      f4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = lrelu(fmaf(a2, yv[q] - m2, b2) + fmaf(ar, rv[q] - mr, br));
      stv4(op + i, o);
      yv = yn;
      rv = rn;
    }
  } else {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < S; i += gridDim.x * 256)
      st1(op + i, lrelu(fmaf(a2, ld1(yp + i) - m2, b2) +
                        fmaf(ar, (rk ? mul_rn(rks, ld1(rp + i)) : ld1(rp + i)) - mr, br)));
  }
}

// The block tail fused with the MaxPool3d(2) that follows it in the encoder (unet3d.py:104-105):
// a thread owns a 2x2x4 input block (two x-adjacent pooling windows), computes its 16 outputs
// (four float4 rows), stores them and the two window maxima (float2) with their argmax bytes.
// Same scan order and comparison as maxpool2_fwd_v_kernel (misc.hip).  Needs even D, H and
// W % 4 == 0.
template <typename T, bool HAS_SRC, bool RK = false>
__global__ __launch_bounds__(256) void norm_act_pool_fwd_kernel(
    const T* __restrict__ y2, long long y2ns, const float* __restrict__ rec2, l3u_norm_src src2,
    const T* __restrict__ r, long long rns, const float* __restrict__ recr, l3u_norm_src srcr,
    int shortcut, T* __restrict__ out, long long ons, T* __restrict__ pooled,
    long long pns, unsigned char* __restrict__ idx, int C, int D, int H, int W) {
  L3U_STAMP_SCOPE(303);
  kargs_now(y2, y2ns, rec2, r, rns, recr, shortcut, out, ons, pooled, pns, idx, C, D, H, W);
  __shared__ float sh[16];
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const long long S = (long long)D * H * W;
  const int Ho = H / 2, W4 = W / 4;
  const long long So = (long long)(D / 2) * Ho * (W / 2), Sp = So / 2;
  constexpr bool rk = RK;   // rank-1 residual (rns < 0): record_r[7] * one stored channel
  const T* yp = y2 + (long long)n * y2ns + (long long)c * S;
  const T* rp = r + (long long)n * (rk ? -rns : rns) + (rk ? 0ll : (long long)c * S);
  T* op = out + (long long)n * ons + (long long)c * S;
  T* pp = pooled + (long long)n * pns + (long long)c * So;
  unsigned short* ip = reinterpret_cast<unsigned short*>(idx + (long long)nc * So);
  auto base_of = [&](long long o) {
    const int q = (int)(o % W4), t = (int)(o / W4), oy = t % Ho, oz = t / Ho;
    return ((long long)(2 * oz) * H + 2 * oy) * W + 4 * q;
  };
  // the records' partial sums are requested first, then the thread's first 2x2x4 block (one round
  // trip for both); every later block one iteration ahead
  const long long o0 = blockIdx.x * 256ll + threadIdx.x, ostep = (long long)gridDim.x * 256;
  f4 yv[4], rv[4];
  auto fetch = [&](long long o) {
    const long long base = base_of(o < Sp ? o : Sp - 1);   // past the end: the last block (cached)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long off = base + ((long long)(j >> 1) * H + (j & 1)) * W;
      yv[j] = ldv4(yp + off);
      rv[j] = ldv4(rp + off);
    }
  };
  RecPre rpre;   // the records' loads before the tile's (common.h block_record2_pre)
  if (HAS_SRC) block_record2_pre(src2, srcr, shortcut != 0, n, c, C, rpre);
  fetch(o0);   // clamped in fetch: no branch ahead of the loads
  float m2, a2, b2, ar = 1.f, br = 0.f, mr = 0.f, rks = 1.f;
  if (HAS_SRC) {
    block_record2_fin(src2, srcr, shortcut != 0, n, c, C, blockIdx.x == 0, sh, rpre);
    m2 = sh[0]; a2 = sh[2]; b2 = sh[3];
    if (shortcut) { mr = sh[8]; ar = sh[10]; br = sh[11]; rks = sh[15]; }
  } else {
    m2 = rec2[(long long)nc * kRec + 0];
    a2 = rec2[(long long)nc * kRec + 2];
    b2 = rec2[(long long)nc * kRec + 3];
    if (shortcut) {
      mr = recr[(long long)nc * kRec + 0];
      ar = recr[(long long)nc * kRec + 2];
      br = recr[(long long)nc * kRec + 3];
      rks = recr[(long long)nc * kRec + 7];
    }
  }
  for (long long o = o0; o < Sp; o += ostep) {
    const long long base = base_of(o);
    f4 v[4];
    if (rk) {
#pragma unroll
      for (int j = 0; j < 4; ++j) rv[j] = mul_rn(rv[j], rks);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = lrelu(fmaf(a2, yv[j][e] - m2, b2) + fmaf(ar, rv[j][e] - mr, br));
    fetch(o + ostep);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long off = base + ((long long)(j >> 1) * H + (j & 1)) * W;
      stv4(op + off, v[j]);
      // the pooled maxima are taken over the values as stored (bf16: rounded), so that the
      // pooled tensor equals MaxPool3d of `out`
      v[j] = round_to(v[j], (const T*)nullptr);
    }
    float b0 = v[0][0], b1 = v[0][2];
    int i0 = 0, i1 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        if (j == 0 && dx == 0) continue;
        const float u0 = v[j][dx], u1 = v[j][2 + dx];
        if (u0 > b0 || u0 != u0) { b0 = u0; i0 = 2 * j + dx; }
        if (u1 > b1 || u1 != u1) { b1 = u1; i1 = 2 * j + dx; }
      }
    stv2(pp + 2 * o, f2_t{b0, b1});
    ip[o] = (unsigned short)(i0 | (i1 << 8));
  }
}

// partials per (c, n, block): [sum g, sum g*xhat2, sum g*xhat_r],  g = dout * lrelu'(out)
#ifndef L3U_NABR_U
#define L3U_NABR_U 2
#endif
constexpr int kNabrU = L3U_NABR_U;   // grid-stride tiles in flight per thread
template <typename T, bool VEC, bool RK = false, bool PL = false>
__global__ __launch_bounds__(256) void norm_act_bwd_reduce_kernel(
    const float* __restrict__ dout, long long dns, const T* __restrict__ out, long long ons,
    const T* __restrict__ y2, long long y2ns, const float* __restrict__ rec2,
    const T* __restrict__ r, long long rns, const float* __restrict__ recr,
    double* __restrict__ part, int N, int C, int S, const float* __restrict__ dscale = nullptr,
    const float* __restrict__ dpool = nullptr, long long dpns = 0,
    const unsigned char* __restrict__ pidx = nullptr, int H = 0, int W = 0) {
  L3U_STAMP_SCOPE(304);
  kargs_now(dout, dns, out, ons, y2, y2ns, rec2, r, rns, recr, part, N, C, S, dscale, dpool, dpns,
            pidx, H, W);
  __shared__ double red[4];
  const int nc = blockIdx.y, c = nc % C, n = nc / C, nb = gridDim.x;
  const float m2 = rec2[(long long)nc * kRec + 0], rs2 = rec2[(long long)nc * kRec + 1];
  float mr = 0.f, rsr = 1.f, rks = 1.f;
  if (recr) {
    mr = recr[(long long)nc * kRec + 0]; rsr = recr[(long long)nc * kRec + 1];
    rks = recr[(long long)nc * kRec + 7];
  }
  constexpr bool rk = RK;   // rank-1 residual (rns < 0): record_r[7] * one stored channel
  const long long co = (long long)c * S;
  // dscale: rank-1 dout = dscale[c] * dz (dz one channel, l3u_outconv_bwd_dz)
  const float* dp = dout + (long long)n * dns + (dscale ? 0 : co);
  const float dsc = dscale ? dscale[c] : 1.f;
  const T* op = out + (long long)n * ons + co;
  const T* yp = y2 + (long long)n * y2ns + co;
  const T* rp = r + (long long)n * (rk ? -rns : rns) + (rk ? 0ll : co);
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  if (VEC) {
    // U grid-stride tiles per round: all their loads in flight before the first use, the sums
    // still taken tile by tile in index order (same bits as one tile per round)
    // Branch-free requests: tail tiles clamped to the last in-range tile (loaded, not summed), the
    // residual read from `out` when there is none, the pooled taps (PL) issued after the tiles; so
    // no load waits on a branch join (guide §6: one vmcnt wait per round, not one per operand).
    constexpr int U = kNabrU;
    const int step = nb * 1024;
    const T* rq = recr ? rp : op;
    for (int i0 = (blockIdx.x * 256 + threadIdx.x) * 4; i0 < S; i0 += U * step) {
      f4 ov[U], dv[U], yv[U], rv[U];
      UnpoolTap pt[U];
      int zz[U], yy[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u * step, S - 4);
        ov[u] = ldv4(op + i);
        dv[u] = ldv4(dp + i);
        yv[u] = ldv4(yp + i);
        rv[u] = ldv4(rq + i);
      }
      if constexpr (PL) {   // + the MaxPool3d backward of the next level (l3u_maxpool2_bwd folded in)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = min(i0 + u * step, S - 4);
          const int HW = H * W, z = fdiv(i, HW, 1.f / HW), rm = i - z * HW, y = fdiv(rm, W, 1.f / W);
          zz[u] = z; yy[u] = y;
          pt[u] = unpool_tap(dpool + (long long)n * dpns + (long long)c * (S / 8),
                             pidx + (long long)nc * (S / 8), z, y, rm - y * W, H, W);
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // every request above issued before the first use
#pragma unroll
      for (int u = 0; u < U; ++u) {
        dv[u] = dsc * dv[u];   // dsc = 1 without dscale: exact
        if constexpr (PL) dv[u] = unpool_apply(dv[u], pt[u], zz[u], yy[u]);
        if (rk) rv[u] = mul_rn(rv[u], rks);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool in = u == 0 || i0 + u * step < S;   // a clamped tail tile: selected away, not branched
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float g = dv[u][q] * lrelu_d(ov[u][q]);
          const double t1 = (double)g * ((yv[u][q] - m2) * rs2);
          const double t2 = (double)g * ((rv[u][q] - mr) * rsr);
          s0 = in ? s0 + g : s0;
          s1 = in ? s1 + t1 : s1;
          if (recr) s2 = in ? s2 + t2 : s2;
        }
      }
    }
  } else {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < S; i += nb * 256) {
      const float g = (dscale ? dsc * ld1(dp + i) : ld1(dp + i)) * lrelu_d(ld1(op + i));
      s0 += g;
      s1 += (double)g * ((ld1(yp + i) - m2) * rs2);
      if (recr) s2 += (double)g * (((rk ? mul_rn(rks, ld1(rp + i)) : ld1(rp + i)) - mr) * rsr);
    }
  }
  s0 = block_sum256d(s0, red);
  s1 = block_sum256d(s1, red);
  s2 = block_sum256d(s2, red);
  if (threadIdx.x == 0) {
    double* o = part + (((long long)c * N + n) * nb + blockIdx.x) * 3;
    o[0] = s0; o[1] = s1; o[2] = s2;
  }
}

// dy2 = rstd2*g2*(g - M0 - xhat2*M1);  dr = shortcut ? rstd_r*g_r*(g - M0 - xhat_r*M2) : g
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void norm_act_bwd_apply_kernel(
    const float* __restrict__ dout, long long dns, const T* __restrict__ out, long long ons,
    const T* __restrict__ y2, long long y2ns, const float* __restrict__ rec2,
    const T* __restrict__ r, long long rns, const float* __restrict__ recr,
    const double* __restrict__ part, int npart, float* __restrict__ dy2, long long dy2ns,
    float* __restrict__ dr, long long drns, int N, int C, int S) {
  L3U_STAMP_SCOPE(305);
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const double* pp = part + ((long long)c * N + n) * npart * 3;
  double t[3];
  seq_sum<3>(pp, npart, t);
  const double t0 = t[0], t1 = t[1], t2 = t[2];
  const float M0 = (float)(t0 / S), M1 = (float)(t1 / S), M2 = (float)(t2 / S);
  const float* q2 = rec2 + (long long)nc * kRec;
  const float mu2 = q2[0], rs2 = q2[1], f2 = q2[1] * q2[5];
  float mur = 0.f, rsr = 1.f, fr = 1.f;
  if (recr) { const float* qr = recr + (long long)nc * kRec; mur = qr[0]; rsr = qr[1]; fr = qr[1] * qr[5]; }
  const long long co = (long long)c * S;
  const float* dp = dout + (long long)n * dns + co;
  const T* op = out + (long long)n * ons + co;
  const T* yp = y2 + (long long)n * y2ns + co;
  const T* rp = r + (long long)n * rns + co;
  float* d2 = dy2 + (long long)n * dy2ns + co;
  float* drp = dr + (long long)n * drns + co;
  if (VEC) {
    for (int i = (blockIdx.x * 256 + threadIdx.x) * 4; i < S; i += gridDim.x * 1024) {
      const f4 dv = ldv4(dp + i), ov = ldv4(op + i);
      const f4 yv = ldv4(yp + i);
      f4 rv = f4{0.f, 0.f, 0.f, 0.f};
      if (recr) rv = ldv4(rp + i);
      f4 o2, orr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float g = dv[q] * lrelu_d(ov[q]);
        o2[q] = f2 * (g - M0 - (yv[q] - mu2) * rs2 * M1);
        orr[q] = recr ? fr * (g - M0 - (rv[q] - mur) * rsr * M2) : g;
      }
      stv4(d2 + i, o2);
      stv4(drp + i, orr);
    }
  } else {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < S; i += gridDim.x * 256) {
      const float g = ld1(dp + i) * lrelu_d(ld1(op + i));
      st1(d2 + i, f2 * (g - M0 - (ld1(yp + i) - mu2) * rs2 * M1));
      st1(drp + i, recr ? fr * (g - M0 - (ld1(rp + i) - mur) * rsr * M2) : g);
    }
  }
}

// Both phases in one launch for planes that one workgroup covers (l3u_norm_act_nblocks(S) == 1:
// the 12^3 / 6^3 levels, where a launch costs more than the work): the three plane sums are
// workgroup sums held by every thread, stored as the single partial, then applied.  Same values,
// bit for bit, as the reduce + apply pair (the apply's fixed-order merge of one partial is exact).
template <typename T, bool VEC, bool PL = false>
__global__ __launch_bounds__(256) void norm_act_bwd_one_kernel(
    const float* __restrict__ dout, long long dns, const T* __restrict__ out, long long ons,
    const T* __restrict__ y2, long long y2ns, const float* __restrict__ rec2,
    const T* __restrict__ r, long long rns, const float* __restrict__ recr,
    double* __restrict__ part, float* __restrict__ dy2, long long dy2ns, float* __restrict__ dr,
    long long drns, int N, int C, int S, const float* __restrict__ dpool = nullptr,
    long long dpns = 0, const unsigned char* __restrict__ pidx = nullptr, int H = 0, int W = 0) {
  L3U_STAMP_SCOPE(306);
  kargs_now(dout, dns, out, ons, y2, y2ns, rec2, r, rns, recr, part, dy2, dy2ns, dr, drns, N, C, S,
            dpool, dpns, pidx, H, W);
  __shared__ double red[4];
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const float* q2 = rec2 + (long long)nc * kRec;
  const float m2 = q2[0], rs2 = q2[1], f2 = q2[1] * q2[5];
  float mr = 0.f, rsr = 1.f, fr = 1.f;
  if (recr) { const float* qr = recr + (long long)nc * kRec; mr = qr[0]; rsr = qr[1]; fr = qr[1] * qr[5]; }
  const long long co = (long long)c * S;
  const float* dp = dout + (long long)n * dns + co;
  const T* op = out + (long long)n * ons + co;
  const T* yp = y2 + (long long)n * y2ns + co;
  const T* rp = r + (long long)n * rns + co;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  float* d2 = dy2 + (long long)n * dy2ns + co;
  float* drp = dr + (long long)n * drns + co;
  constexpr int NI = 2;   // S <= NI * 1024 (the 12^3 and 6^3 levels): operands held in registers
  if (VEC && S <= NI * 1024) {
    // every tile requested at once, one load phase; the apply reuses the registers (same
    // per-thread order and expressions as the looped form below: same bits)
    // (clamped, branch-free requests as in norm_act_bwd_reduce_kernel; the pooled taps last)
    f4 dv[NI], ov[NI], yv[NI], rv[NI];
    UnpoolTap pt[NI];
    int zz[NI], yy[NI];
    const T* rq = recr ? rp : op;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = min(threadIdx.x * 4 + k * 1024, S - 4);
      dv[k] = ldv4(dp + i);
      ov[k] = ldv4(op + i);
      yv[k] = ldv4(yp + i);
      rv[k] = ldv4(rq + i);
    }
    if (PL) {   // + the next level's MaxPool3d backward (l3u_maxpool2_bwd folded in)
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        const int i = min(threadIdx.x * 4 + k * 1024, S - 4);
        const int HW = H * W, z = fdiv(i, HW, 1.f / HW), rm = i - z * HW, y = fdiv(rm, W, 1.f / W);
        zz[k] = z; yy[k] = y;
        pt[k] = unpool_tap(dpool + (long long)n * dpns + (long long)c * (S / 8),
                           pidx + (long long)nc * (S / 8), z, y, rm - y * W, H, W);
      }
#pragma unroll
      for (int k = 0; k < NI; ++k) dv[k] = unpool_apply(dv[k], pt[k], zz[k], yy[k]);
    }
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      // (a branch, not a select as in the reduce: g recomputed in the apply below then contracts
      // exactly as in norm_act_bwd_apply_kernel -- the two stay bit-identical; the loads above
      // are used after the branch too, so they cannot sink into it)
      if (threadIdx.x * 4 + k * 1024 < S) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float g = dv[k][q] * lrelu_d(ov[k][q]);
          s0 += g;
          s1 += (double)g * ((yv[k][q] - m2) * rs2);
          if (recr) s2 += (double)g * ((rv[k][q] - mr) * rsr);
        }
      }
    }
    s0 = block_sum256d(s0, red);
    s1 = block_sum256d(s1, red);
    s2 = block_sum256d(s2, red);
    if (threadIdx.x == 0) {
      double* o = part + ((long long)c * N + n) * 3;
      o[0] = s0; o[1] = s1; o[2] = s2;
    }
    const float M0 = (float)((0.0 + s0) / S), M1 = (float)((0.0 + s1) / S), M2 = (float)((0.0 + s2) / S);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = threadIdx.x * 4 + k * 1024;
      if (i < S) {
        f4 o2, orr;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float g = dv[k][q] * lrelu_d(ov[k][q]);
          o2[q] = f2 * (g - M0 - (yv[k][q] - m2) * rs2 * M1);
          orr[q] = recr ? fr * (g - M0 - (rv[k][q] - mr) * rsr * M2) : g;
        }
        stv4(d2 + i, o2);
        stv4(drp + i, orr);
      }
    }
    return;
  }
  if (VEC) {
    for (int i = threadIdx.x * 4; i < S; i += 1024) {
      const f4 dv = ldv4(dp + i), ov = ldv4(op + i);
      const f4 yv = ldv4(yp + i);
      f4 rv = f4{0.f, 0.f, 0.f, 0.f};
      if (recr) rv = ldv4(rp + i);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float g = dv[q] * lrelu_d(ov[q]);
        s0 += g;
        s1 += (double)g * ((yv[q] - m2) * rs2);
        if (recr) s2 += (double)g * ((rv[q] - mr) * rsr);
      }
    }
  } else {
    for (int i = threadIdx.x; i < S; i += 256) {
      const float g = ld1(dp + i) * lrelu_d(ld1(op + i));
      s0 += g;
      s1 += (double)g * ((ld1(yp + i) - m2) * rs2);
      if (recr) s2 += (double)g * ((ld1(rp + i) - mr) * rsr);
    }
  }
  s0 = block_sum256d(s0, red);
  s1 = block_sum256d(s1, red);
  s2 = block_sum256d(s2, red);
  if (threadIdx.x == 0) {
    double* o = part + ((long long)c * N + n) * 3;
    o[0] = s0; o[1] = s1; o[2] = s2;
  }
  const float M0 = (float)((0.0 + s0) / S), M1 = (float)((0.0 + s1) / S), M2 = (float)((0.0 + s2) / S);
  if (VEC) {
    for (int i = threadIdx.x * 4; i < S; i += 1024) {
      const f4 dv = ldv4(dp + i), ov = ldv4(op + i);
      const f4 yv = ldv4(yp + i);
      f4 rv = f4{0.f, 0.f, 0.f, 0.f};
      if (recr) rv = ldv4(rp + i);
      f4 o2, orr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float g = dv[q] * lrelu_d(ov[q]);
        o2[q] = f2 * (g - M0 - (yv[q] - m2) * rs2 * M1);
        orr[q] = recr ? fr * (g - M0 - (rv[q] - mr) * rsr * M2) : g;
      }
      stv4(d2 + i, o2);
      stv4(drp + i, orr);
    }
  } else {
    for (int i = threadIdx.x; i < S; i += 256) {
      const float g = ld1(dp + i) * lrelu_d(ld1(op + i));
      st1(d2 + i, f2 * (g - M0 - (ld1(yp + i) - m2) * rs2 * M1));
      st1(drp + i, recr ? fr * (g - M0 - (ld1(rp + i) - mr) * rsr * M2) : g);
    }
  }
}

// InstanceNorm backward apply for the inner norm (after dw3_bwd MODE 1 produced dpre + sums):
// dy = rstd*gamma*(dpre - M1 - xhat*M2); in-place allowed (dy == dpre)
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void in_bwd_apply_kernel(
    const float* dpre, long long dns, const T* __restrict__ y, long long yns,
    const float* __restrict__ rec, const double* __restrict__ part, int npart, float* dy,
    long long dyns, int N, int C, int S) {
  L3U_STAMP_SCOPE(307);
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const double* pp = part + ((long long)c * N + n) * npart * 2;
  // the partial sums over the workgroup's threads (i = tid, tid + 256, ...) and a fixed-order
  // block sum: one or two memory round trips for the 432 per-block partials of a 48^3 grouped
  // conv, where an in-order sum took 54 dependent rounds (54 us at [4,16,48^3])
  __shared__ double red[4];
  double a0 = 0.0, a1 = 0.0;
  for (int i = threadIdx.x; i < npart; i += 256) {
    a0 += pp[2 * i];
    a1 += pp[2 * i + 1];
  }
  const double t0 = block_sum256d(a0, red), t1 = block_sum256d(a1, red);
  const float M1 = (float)(t0 / S), M2 = (float)(t1 / S);
  const float* q = rec + (long long)nc * kRec;
  const float mu = q[0], rs = q[1], f = q[1] * q[5];
  const long long co = (long long)c * S;
  const float* dp = dpre + (long long)n * dns + co;
  const T* yp = y + (long long)n * yns + co;
  float* op = dy + (long long)n * dyns + co;
  if (VEC) {
    for (int i = (blockIdx.x * 256 + threadIdx.x) * 4; i < S; i += gridDim.x * 1024) {
      const f4 dv = ldv4(dp + i), yv = ldv4(yp + i);
      f4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = f * (dv[k] - M1 - (yv[k] - mu) * rs * M2);
      stv4(op + i, o);
    }
  } else {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < S; i += gridDim.x * 256)
      st1(op + i, f * (ld1(dp + i) - M1 - (ld1(yp + i) - mu) * rs * M2));
  }
}

constexpr int kElemPerBlock = 4096;
#ifndef L3U_ELEM_MAXB
#define L3U_ELEM_MAXB 16
#endif
constexpr int kElemMaxBlocks = L3U_ELEM_MAXB;
// workgroups per (n, c) plane of the elementwise IN kernels: few enough that the per-workgroup
// record merge (in-kernel finalize) stays small next to the streaming work
int elem_blocks(int S) {
  int b = (S + kElemPerBlock - 1) / kElemPerBlock;
  return b > kElemMaxBlocks ? kElemMaxBlocks : (b < 1 ? 1 : b);
}

// the forward block tails (no partials, so free to differ from elem_blocks): workgroups per plane
#ifndef L3U_NAF_ELEMS
#define L3U_NAF_ELEMS 4096
#endif
#ifndef L3U_NAF_MAXB
#define L3U_NAF_MAXB 16
#endif
int fwd_blocks(int S) {
  int b = (S + L3U_NAF_ELEMS - 1) / L3U_NAF_ELEMS;
  return b > L3U_NAF_MAXB ? L3U_NAF_MAXB : (b < 1 ? 1 : b);
}

}  // namespace

extern "C" {

int l3u_in_finalize(const float* stat_part, int nsb, const float* gamma, const float* beta,
                    float drop_p, unsigned long long seed, const int* step, int layer, float* rec,
                    int N, int C, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && nsb > 0 && drop_p >= 0.f && drop_p < 1.f && rec != nullptr);
  const int NC = N * C;
  l3u_norm_src src{stat_part, nsb, layer, gamma, beta, drop_p, seed, step, rec};
  hipLaunchKernelGGL(in_finalize_kernel, dim3((NC + 3) / 4), dim3(256), 0, stream, src, NC, C);
  L3U_CHECK_LAUNCH();
}

int l3u_norm_act_nblocks(int S) { return elem_blocks(S); }

}  // extern "C"

namespace {

template <typename T>
int norm_act_fwd_impl(const T* y2, long long y2_nstride, const float* rec2,
                      const l3u_norm_src* src2, const T* r, long long r_nstride,
                      const float* rec_r, const l3u_norm_src* src_r, int shortcut, T* out,
                      long long out_nstride, int N, int C, int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0);
  L3U_REQUIRE(src2 ? (!shortcut || src_r) : (rec2 && (!shortcut || rec_r)));
  const bool vec = S % 4 == 0 && y2_nstride % 4 == 0 && r_nstride % 4 == 0 && out_nstride % 4 == 0;
  L3U_REQUIRE(r_nstride >= 0 || (sizeof(T) == 4 && shortcut && vec));   // rank-1 r: fp32 Conv1x1 shortcut
  dim3 grid(fwd_blocks(S), N * C);
  const l3u_norm_src z{};
  const l3u_norm_src s2 = src2 ? *src2 : z, sr = src_r ? *src_r : z;
#define NAF0(V_, S_, R_) hipLaunchKernelGGL((norm_act_fwd_kernel<T, V_, S_, R_>), grid, dim3(256), 0, stream, y2, \
      y2_nstride, rec2, s2, r, r_nstride, rec_r, sr, shortcut, out, out_nstride, C, S)
#define NAF(V_, S_) NAF0(V_, S_, false)
  if (r_nstride < 0) { if constexpr (sizeof(T) == 4) { if (src2) NAF0(true, true, true); else NAF0(true, false, true); } }
  else if (src2) { if (vec) NAF(true, true); else NAF(false, true); }
  else { if (vec) NAF(true, false); else NAF(false, false); }
#undef NAF
#undef NAF0
  L3U_CHECK_LAUNCH();
}

template <typename T>
int norm_act_pool_fwd_impl(const T* y2, long long y2_nstride, const float* rec2,
                           const l3u_norm_src* src2, const T* r, long long r_nstride,
                           const float* rec_r, const l3u_norm_src* src_r, int shortcut, T* out,
                           long long out_nstride, T* pooled, long long pooled_nstride,
                           unsigned char* idx, int N, int C, int D, int H, int W,
                           hipStream_t stream) {
  constexpr int E = (int)sizeof(T);
  L3U_REQUIRE(N > 0 && C > 0 && D >= 2 && H >= 2 && W >= 4);
  L3U_REQUIRE(src2 ? (!shortcut || src_r) : (rec2 && (!shortcut || rec_r)));
  L3U_REQUIRE(r_nstride >= 0 || (sizeof(T) == 4 && shortcut));   // rank-1 r: fp32 Conv1x1 shortcut
  L3U_REQUIRE(!(D & 1) && !(H & 1) && !(W & 3) && y2_nstride % 4 == 0 && r_nstride % 4 == 0 &&
              out_nstride % 4 == 0 && pooled_nstride % 2 == 0 && ((uintptr_t)y2 & (4 * E - 1)) == 0 &&
              ((uintptr_t)r & (4 * E - 1)) == 0 && ((uintptr_t)out & (4 * E - 1)) == 0 &&
              ((uintptr_t)pooled & (2 * E - 1)) == 0 && ((uintptr_t)idx & 1) == 0);
  const long long S = (long long)D * H * W;
  dim3 grid(fwd_blocks((int)S), N * C);
  const l3u_norm_src z{};
  const l3u_norm_src s2 = src2 ? *src2 : z, sr = src_r ? *src_r : z;
#define NAP(S_, R_) hipLaunchKernelGGL((norm_act_pool_fwd_kernel<T, S_, R_>), grid, dim3(256), 0, stream, y2, \
      y2_nstride, rec2, s2, r, r_nstride, rec_r, sr, shortcut, out, out_nstride, pooled, \
      pooled_nstride, idx, C, D, H, W)
  if (r_nstride < 0) { if constexpr (sizeof(T) == 4) { if (src2) NAP(true, true); else NAP(false, true); } }
  else if (src2) NAP(true, false);
  else NAP(false, false);
#undef NAP
  L3U_CHECK_LAUNCH();
}

template <typename T>
int norm_act_bwd_reduce_impl(const float* dout, long long dout_nstride, const T* out,
                             long long out_nstride, const T* y2, long long y2_nstride,
                             const float* rec2, const T* r, long long r_nstride,
                             const float* rec_r, double* part, int N, int C, int S,
                             hipStream_t stream, const float* dscale = nullptr,
                             const float* dpool = nullptr, long long dpns = 0,
                             const unsigned char* pidx = nullptr, int H = 0, int W = 0) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0);
  L3U_REQUIRE(r_nstride >= 0 || (sizeof(T) == 4 && rec_r != nullptr));   // rank-1 r: fp32 only
  const bool vec = S % 4 == 0 && dout_nstride % 4 == 0 && out_nstride % 4 == 0 &&
                   y2_nstride % 4 == 0 && r_nstride % 4 == 0;
  L3U_REQUIRE(dpool == nullptr || (vec && pidx && H % 2 == 0 && W % 4 == 0 && (S / (H * W)) % 2 == 0 &&
                                   dpns % 2 == 0 && ((uintptr_t)dpool & 7) == 0));
  dim3 grid(elem_blocks(S), N * C);
  L3U_REQUIRE(r_nstride >= 0 || vec);
#define NABR(RK_, PL_) hipLaunchKernelGGL((norm_act_bwd_reduce_kernel<T, true, RK_, PL_>), grid, dim3(256), 0, \
      stream, dout, dout_nstride, out, out_nstride, y2, y2_nstride, rec2, r, r_nstride, rec_r, part, N, C, S, \
      dscale, dpool, dpns, pidx, H, W)
  if (r_nstride < 0) {
    if constexpr (sizeof(T) == 4) { if (dpool) NABR(true, true); else NABR(true, false); }
  } else if (vec) { if (dpool) NABR(false, true); else NABR(false, false); }
#undef NABR
  else hipLaunchKernelGGL((norm_act_bwd_reduce_kernel<T, false>), grid, dim3(256), 0, stream, dout, dout_nstride, out, out_nstride, y2, y2_nstride, rec2, r, r_nstride, rec_r, part, N, C, S, dscale);
  L3U_CHECK_LAUNCH();
}

template <typename T>
int norm_act_bwd_apply_impl(const float* dout, long long dout_nstride, const T* out,
                            long long out_nstride, const T* y2, long long y2_nstride,
                            const float* rec2, const T* r, long long r_nstride,
                            const float* rec_r, const double* part, float* dy2,
                            long long dy2_nstride, float* dr, long long dr_nstride, int N, int C,
                            int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0);
  L3U_REQUIRE(r_nstride >= 0);   // no rank-1 residual on the split tail
  const bool vec = S % 4 == 0 && dout_nstride % 4 == 0 && out_nstride % 4 == 0 &&
                   y2_nstride % 4 == 0 && r_nstride % 4 == 0 && dy2_nstride % 4 == 0 &&
                   dr_nstride % 4 == 0;
  const int npart = elem_blocks(S);
  dim3 grid(npart, N * C);
  if (vec) hipLaunchKernelGGL((norm_act_bwd_apply_kernel<T, true>), grid, dim3(256), 0, stream, dout, dout_nstride, out, out_nstride, y2, y2_nstride, rec2, r, r_nstride, rec_r, part, npart, dy2, dy2_nstride, dr, dr_nstride, N, C, S);
  else hipLaunchKernelGGL((norm_act_bwd_apply_kernel<T, false>), grid, dim3(256), 0, stream, dout, dout_nstride, out, out_nstride, y2, y2_nstride, rec2, r, r_nstride, rec_r, part, npart, dy2, dy2_nstride, dr, dr_nstride, N, C, S);
  L3U_CHECK_LAUNCH();
}

template <typename T>
int norm_act_bwd_impl(const float* dout, long long dout_nstride, const T* out,
                      long long out_nstride, const T* y2, long long y2_nstride,
                      const float* rec2, const T* r, long long r_nstride, const float* rec_r,
                      double* part, float* dy2, long long dy2_nstride, float* dr,
                      long long dr_nstride, int N, int C, int S, hipStream_t stream,
                      const float* dpool = nullptr, long long dpns = 0,
                      const unsigned char* pidx = nullptr, int D = 0, int H = 0, int W = 0) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0 && elem_blocks(S) == 1);
  L3U_REQUIRE(r_nstride >= 0);   // no rank-1 residual on the split tail
  const bool vec = S % 4 == 0 && dout_nstride % 4 == 0 && out_nstride % 4 == 0 &&
                   y2_nstride % 4 == 0 && r_nstride % 4 == 0 && dy2_nstride % 4 == 0 &&
                   dr_nstride % 4 == 0;
  // the folded MaxPool3d backward: the register-held form (S <= 2048), even D / H, W % 4 == 0
  L3U_REQUIRE(dpool == nullptr || (vec && pidx && S <= 2048 && D * H * W == S && D % 2 == 0 &&
                                   H % 2 == 0 && W % 4 == 0 && dpns % 2 == 0 &&
                                   ((uintptr_t)dpool & 7) == 0));
  dim3 grid(1, N * C);
  if (vec && dpool) hipLaunchKernelGGL((norm_act_bwd_one_kernel<T, true, true>), grid, dim3(256), 0, stream, dout, dout_nstride, out, out_nstride, y2, y2_nstride, rec2, r, r_nstride, rec_r, part, dy2, dy2_nstride, dr, dr_nstride, N, C, S, dpool, dpns, pidx, H, W);
  else if (vec) hipLaunchKernelGGL((norm_act_bwd_one_kernel<T, true>), grid, dim3(256), 0, stream, dout, dout_nstride, out, out_nstride, y2, y2_nstride, rec2, r, r_nstride, rec_r, part, dy2, dy2_nstride, dr, dr_nstride, N, C, S);
  else hipLaunchKernelGGL((norm_act_bwd_one_kernel<T, false>), grid, dim3(256), 0, stream, dout, dout_nstride, out, out_nstride, y2, y2_nstride, rec2, r, r_nstride, rec_r, part, dy2, dy2_nstride, dr, dr_nstride, N, C, S);
  L3U_CHECK_LAUNCH();
}

template <typename T>
int in_bwd_apply_impl(const float* dpre, long long dpre_nstride, const T* y, long long y_nstride,
                      const float* rec, const double* in_part, int npart, float* dy,
                      long long dy_nstride, int N, int C, int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0 && npart > 0);
  const bool vec = S % 4 == 0 && dpre_nstride % 4 == 0 && y_nstride % 4 == 0 && dy_nstride % 4 == 0;
  dim3 grid(elem_blocks(S), N * C);
  if (vec) hipLaunchKernelGGL((in_bwd_apply_kernel<T, true>), grid, dim3(256), 0, stream, dpre, dpre_nstride, y, y_nstride, rec, in_part, npart, dy, dy_nstride, N, C, S);
  else hipLaunchKernelGGL((in_bwd_apply_kernel<T, false>), grid, dim3(256), 0, stream, dpre, dpre_nstride, y, y_nstride, rec, in_part, npart, dy, dy_nstride, N, C, S);
  L3U_CHECK_LAUNCH();
}

}  // namespace

// ---- C-ABI: fp32 entry points and their _bf16 twins (include/l3u.h) ----------------------------
#define P_NAF(TT) (const TT* y2, long long y2_nstride, const float* rec2, const l3u_norm_src* src2, \
    const TT* r, long long r_nstride, const float* rec_r, const l3u_norm_src* src_r, int shortcut,  \
    TT* out, long long out_nstride, int N, int C, int S, hipStream_t stream)
L3U_TWIN(l3u_norm_act_fwd, P_NAF, norm_act_fwd_impl(bp(y2), y2_nstride, rec2, src2, bp(r), r_nstride,
         rec_r, src_r, shortcut, bp(out), out_nstride, N, C, S, stream))
#define P_NAP(TT) (const TT* y2, long long y2_nstride, const float* rec2, const l3u_norm_src* src2, \
    const TT* r, long long r_nstride, const float* rec_r, const l3u_norm_src* src_r, int shortcut,  \
    TT* out, long long out_nstride, TT* pooled, long long pooled_nstride, unsigned char* idx, int N, \
    int C, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_norm_act_pool_fwd, P_NAP, norm_act_pool_fwd_impl(bp(y2), y2_nstride, rec2, src2, bp(r),
         r_nstride, rec_r, src_r, shortcut, bp(out), out_nstride, bp(pooled), pooled_nstride, idx, N,
         C, D, H, W, stream))
#define P_NBR(TT) (const float* dout, long long dout_nstride, const TT* out, long long out_nstride,   \
    const TT* y2, long long y2_nstride, const float* rec2, const TT* r, long long r_nstride,        \
    const float* rec_r, double* part, int N, int C, int S, hipStream_t stream)
L3U_TWIN(l3u_norm_act_bwd_reduce, P_NBR, norm_act_bwd_reduce_impl(dout, dout_nstride, bp(out),
         out_nstride, bp(y2), y2_nstride, rec2, bp(r), r_nstride, rec_r, part, N, C, S, stream))
// rank-1 output gradient dout[c] = dscale[c] * dz (dz: one channel, batch stride dz_nstride)
#define P_NBR1(TT) (const float* dz, long long dz_nstride, const float* dscale, const TT* out,        \
    long long out_nstride, const TT* y2, long long y2_nstride, const float* rec2, const TT* r,       \
    long long r_nstride, const float* rec_r, double* part, int N, int C, int S, hipStream_t stream)
// the block-output gradient = skip gradient + the next level's MaxPool3d backward, folded in
#define P_NBRU(TT) (const float* dskip, long long dskip_nstride, const float* dpool,                  \
    long long dpool_nstride, const unsigned char* idx, const TT* out, long long out_nstride,         \
    const TT* y2, long long y2_nstride, const float* rec2, const TT* r, long long r_nstride,        \
    const float* rec_r, double* part, int N, int C, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_norm_act_bwd_reduce_up, P_NBRU, dpool == nullptr ? (int)hipErrorInvalidValue :
         norm_act_bwd_reduce_impl(dskip, dskip_nstride, bp(out), out_nstride, bp(y2), y2_nstride, rec2,
         bp(r), r_nstride, rec_r, part, N, C, D * H * W, stream, nullptr, dpool, dpool_nstride, idx, H,
         W))
L3U_TWIN(l3u_norm_act_bwd_reduce_r1, P_NBR1, dscale == nullptr ? (int)hipErrorInvalidValue :
         norm_act_bwd_reduce_impl(dz, dz_nstride, bp(out), out_nstride, bp(y2), y2_nstride, rec2, bp(r),
         r_nstride, rec_r, part, N, C, S, stream, dscale))
#define P_NBA(TT) (const float* dout, long long dout_nstride, const TT* out, long long out_nstride,   \
    const TT* y2, long long y2_nstride, const float* rec2, const TT* r, long long r_nstride,        \
    const float* rec_r, const double* part, float* dy2, long long dy2_nstride, float* dr,          \
    long long dr_nstride, int N, int C, int S, hipStream_t stream)
L3U_TWIN(l3u_norm_act_bwd_apply, P_NBA, norm_act_bwd_apply_impl(dout, dout_nstride, bp(out),
         out_nstride, bp(y2), y2_nstride, rec2, bp(r), r_nstride, rec_r, part, dy2, dy2_nstride,
         dr, dr_nstride, N, C, S, stream))
#define P_NB1(TT) (const float* dout, long long dout_nstride, const TT* out, long long out_nstride,   \
    const TT* y2, long long y2_nstride, const float* rec2, const TT* r, long long r_nstride,        \
    const float* rec_r, double* part, float* dy2, long long dy2_nstride, float* dr,                 \
    long long dr_nstride,                                                                            \
    int N, int C, int S, hipStream_t stream)
L3U_TWIN(l3u_norm_act_bwd, P_NB1, norm_act_bwd_impl(dout, dout_nstride, bp(out), out_nstride,
         bp(y2), y2_nstride, rec2, bp(r), r_nstride, rec_r, part, dy2, dy2_nstride, dr,
         dr_nstride, N, C, S, stream))
// the same with the block-output gradient = skip gradient + the next level's MaxPool3d backward
// (l3u_maxpool2_bwd folded in, the one-launch planes of l3u_norm_act_bwd)
#define P_NB1U(TT) (const float* dskip, long long dskip_nstride, const float* dpool,                 \
    long long dpool_nstride, const unsigned char* idx, const TT* out, long long out_nstride,         \
    const TT* y2, long long y2_nstride, const float* rec2, const TT* r, long long r_nstride,        \
    const float* rec_r, double* part, float* dy2, long long dy2_nstride, float* dr,                 \
    long long dr_nstride, int N, int C, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_norm_act_bwd_up, P_NB1U, dpool == nullptr ? (int)hipErrorInvalidValue :
         norm_act_bwd_impl(dskip, dskip_nstride, bp(out), out_nstride, bp(y2), y2_nstride, rec2,
         bp(r), r_nstride, rec_r, part, dy2, dy2_nstride, dr, dr_nstride, N, C, D * H * W, stream,
         dpool, dpool_nstride, idx, D, H, W))
#define P_IBA(TT) (const float* dpre, long long dpre_nstride, const TT* y, long long y_nstride,    \
    const float* rec, const double* in_part, int npart, float* dy, long long dy_nstride, int N,      \
    int C,                                                                                           \
    int S, hipStream_t stream)
L3U_TWIN(l3u_in_bwd_apply, P_IBA, in_bwd_apply_impl(dpre, dpre_nstride, bp(y), y_nstride, rec,
         in_part, npart, dy, dy_nstride, N, C, S, stream))
