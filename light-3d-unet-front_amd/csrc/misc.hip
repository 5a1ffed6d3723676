// Remaining hot-path ops:
//   maxpool2_fwd/bwd     nn.MaxPool3d(2, 2)                                   unet3d.py:101
//   outconv fwd/bwd      out_conv 1x1x1 (+bias) + Sigmoid                      unet3d.py:201-202,220-221
//   ftl_*                FocalTverskyLoss forward sums / loss / closed-form backward  losses.py:30-54
//   adamw                torch.optim.AdamW step on the flat parameter buffer     trainer.py:75-79
//   reduce_segments      deterministic second stage of every split-K / partial reduction
#include "common.h"
#ifdef L3U_STAMP
#include <vector>
#endif
using namespace l3u;

typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

// ---------------------------------------------------------------- maxpool 2x2x2 (floor mode)
template <typename T>
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(
    const T* __restrict__ x, long long xns, T* __restrict__ y, long long yns,
    unsigned char* __restrict__ idx, int C, int D, int H, int W) {
  L3U_STAMP_SCOPE(401);
  const int Do = D / 2, Ho = H / 2, Wo = W / 2;
  const long long So = (long long)Do * Ho * Wo, Si = (long long)D * H * W;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const T* xp = x + (long long)n * xns + (long long)c * Si;
  T* yp = y + (long long)n * yns + (long long)c * So;
  unsigned char* ip = idx + (long long)nc * So;
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < So; o += (long long)gridDim.x * 256) {
    const int ox = (int)(o % Wo), t = (int)(o / Wo), oy = t % Ho, oz = t / Ho;
    const T* b = xp + ((long long)(2 * oz) * H + 2 * oy) * W + 2 * ox;
    float best = ld1(b);
    int bi = 0;
    // scan order (dz, dy, dx) and strict '>' (first maximum wins; NaN propagates) as torch CPU
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      const int dz = j >> 2, dy = (j >> 1) & 1, dx = j & 1;
      const float v = ld1(b + ((long long)dz * H + dy) * W + dx);
      if (v > best || v != v) { best = v; bi = j; }
    }
    st1(yp + o, best);
    ip[o] = (unsigned char)bi;
  }
}

// dx = route(dy) (+ add): every input voxel is written exactly once (covers odd-size tails)
template <typename T>
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(
    const T* __restrict__ dy, long long dyns, const unsigned char* __restrict__ idx,
    const T* __restrict__ add, long long addns, T* __restrict__ dx, long long dxns,
    int C, int D, int H, int W) {
  L3U_STAMP_SCOPE(402);
  const int Do = D / 2, Ho = H / 2, Wo = W / 2;
  const long long So = (long long)Do * Ho * Wo, Si = (long long)D * H * W;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const T* dyp = dy + (long long)n * dyns + (long long)c * So;
  const unsigned char* ip = idx + (long long)nc * So;
  const T* ap = add ? add + (long long)n * addns + (long long)c * Si : nullptr;
  T* dxp = dx + (long long)n * dxns + (long long)c * Si;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < Si; i += (long long)gridDim.x * 256) {
    const int xx = (int)(i % W), t = (int)(i / W), yy = t % H, zz = t / H;
    float v = 0.f;
    const int oz = zz >> 1, oy = yy >> 1, ox = xx >> 1;
    if (oz < Do && oy < Ho && ox < Wo) {
      const long long o = ((long long)oz * Ho + oy) * Wo + ox;
      const int j = ((zz & 1) << 2) | ((yy & 1) << 1) | (xx & 1);
      if (ip[o] == j) v = ld1(dyp + o);
    }
    if (ap) v += ld1(ap + i);
    st1(dxp + i, v);
  }
}

// ---------------------------------------------------------------- out_conv + sigmoid
// p = sigmoid(b + sum_c w[c] h[c]); 4 voxels per thread (float4 when VEC).  t != NULL: also the
// FocalTversky partials of this block, ftl_part[n*nb + blk] = {sum p*t, sum p, sum t} (the loss's
// first reduction stage fused into the producer of p: losses.py:40-42).
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void outconv_fwd_kernel(
    const T* __restrict__ h, long long hns, const float* __restrict__ w,
    const float* __restrict__ b, float* __restrict__ p, const float* __restrict__ t,
    float* __restrict__ ftl_part, int C, int S) {
  L3U_STAMP_SCOPE(403);
  __shared__ float red[4];
  const int n = blockIdx.y;
  const T* hp = h + (long long)n * hns;
  float* pp = p + (long long)n * S;
  const int i0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  // the targets are requested with the channels (one round trip for every operand; they were
  // loaded after the probabilities' store)
  f4 tv4 = {0.f, 0.f, 0.f, 0.f};
  if (VEC && t != nullptr && i0 < S) tv4 = ldv4(t + (long long)n * S + i0);
  const float bv = b[0];
  f4 z = {bv, bv, bv, bv};
  if (VEC) {
    // every channel's float4 requested before the first use (C <= 32; the runtime-C loop issued
    // one load per round trip), then added in channel order as before
    f4 hv[32];
#pragma unroll
    for (int c = 0; c < 32; ++c)
      if (c < C && i0 < S) hv[c] = ldv4(hp + (long long)c * S + i0);
#pragma unroll
    for (int c = 0; c < 32; ++c)
      if (c < C && i0 < S) z += w[c] * hv[c];
  } else {
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (i0 + q < S) z[q] = fmaf(w[c], ld1(hp + (long long)c * S + i0 + q), z[q]);
  }
  f4 pv;
#pragma unroll
  for (int q = 0; q < 4; ++q) pv[q] = 1.f / (1.f + expf(-z[q]));
  if (VEC) {
    if (i0 < S) *reinterpret_cast<f4*>(pp + i0) = pv;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (i0 + q < S) pp[i0 + q] = pv[q];
  }
  if (t == nullptr) return;
  float spt = 0.f, sp = 0.f, st = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (i0 + q < S) {
      const float tv = VEC ? tv4[q] : t[(long long)n * S + i0 + q];
      spt = fmaf(pv[q], tv, spt);
      sp += pv[q];
      st += tv;
    }
  }
  spt = block_sum256(spt, red);
  sp = block_sum256(sp, red);
  st = block_sum256(st, red);
  if (threadIdx.x == 0) {
    float* o = ftl_part + ((long long)n * gridDim.x + blockIdx.x) * 3;
    o[0] = spt;
    o[1] = sp;
    o[2] = st;
  }
}

struct FtlCoef { double loss, A, B; };

L3U_DEV FtlCoef ftl_coef(const double* sums, double alpha, double beta, double gamma, double smooth) {
  const double tp = sums[0], fp = sums[1] - sums[0], fn = sums[2] - sums[0];
  const double dn = tp + alpha * fn + beta * fp + smooth;
  const double ti = (tp + smooth) / dn;
  const double one_m = 1.0 - ti;
  FtlCoef r;
  r.loss = pow(one_m, gamma);
  const double pre = -gamma * pow(one_m, gamma - 1.0) / (dn * dn);
  r.A = pre * (dn - (tp + smooth) * (1.0 - alpha));   // t = 1
  r.B = pre * (-(tp + smooth) * beta);                 // t = 0
  return r;
}

// dz = dL/dp * p(1-p); dh[c] = w[c] * dz; part[n*nb + blk][0..C-1] = sum dz*h[c], [C] = sum dz.
// dL/dp comes from dp, or (dp == NULL) from the FocalTversky closed form A t + B (1 - t) of the
// global sums (losses.py:30-54), fused so the loss gradient is never written out.
// The three FocalTversky sums over nb partials {p*t, p, t}: lane-strided fp64 sums, then a fixed
// DPP wave reduction (every lane gets the totals); one 64-lane wave.  l3u_ftl_reduce and the
// in-kernel reduce of l3u_outconv_bwd_ftl share it, so both give the same bits.
L3U_DEV void ftl_lane_sums(const float* __restrict__ part, int nb, double& a, double& b, double& c) {
  const int l = threadIdx.x & 63;
  a = b = c = 0.0;
  // 8 strided partials in flight per lane (one L2 round trip instead of eight), added in the same
  // i order; out-of-range slots add +0.0, which leaves a (never -0.0) unchanged: same bits
  // (clamped unconditional loads, the out-of-range slots dropped by a select at the add: the
  // predicated form `ok ? part[..] : 0` was compiled as a branch around each load with a
  // vmcnt(0) behind it -- eight dependent round trips, behind the streamed operands of the
  // out_conv backward)
  constexpr int B = 8;
  for (int i = l; i < nb; i += B * 64) {
    float va[B], vb[B], vc[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int j = min(i + u * 64, nb - 1);
      va[u] = part[j * 3];
      vb[u] = part[j * 3 + 1];
      vc[u] = part[j * 3 + 2];
    }
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const bool ok = i + u * 64 < nb;
      a += ok ? va[u] : 0.f;
      b += ok ? vb[u] : 0.f;
      c += ok ? vc[u] : 0.f;
    }
  }
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  c = wave_sum_d(c);
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void outconv_bwd_kernel(
    int dz_only, const float* __restrict__ dp, const float* __restrict__ p, const float* __restrict__ t,
    const double* __restrict__ sums, double alpha, double beta, double gamma, double smooth,
    const float* __restrict__ gscale, const T* __restrict__ h, long long hns,
    const float* __restrict__ w, float* __restrict__ dh, long long dhns,
    double* __restrict__ part, float* __restrict__ loss, int C, int S,
    const float* __restrict__ fpart = nullptr, int fnp = 0) {
  L3U_STAMP_SCOPE(404);
  extern __shared__ double redd[];   // [4][C+1]
  const int n = blockIdx.y, nb = gridDim.x;
  const T* hp = h + (long long)n * hns;
  float* dhp = dh + (long long)n * dhns;
  const long long o = (long long)n * S;
  const int i0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  // VEC: the streamed operands (p, t or dp, the C channels of h) are requested first, so their
  // latency overlaps the FocalTversky prologue below
  f4 pv4 = {0.f, 0.f, 0.f, 0.f}, gv4 = {0.f, 0.f, 0.f, 0.f};
  f4 hv[VEC ? 32 : 1];
  if (VEC) {
    if (i0 < S) {
      pv4 = ldv4(p + o + i0);
      gv4 = ldv4((dp ? dp : t) + o + i0);
    }
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      hv[c] = f4{0.f, 0.f, 0.f, 0.f};
      if (c < C && i0 < S) hv[c] = ldv4(hp + (long long)c * S + i0);
    }
  }
  float cA = 0.f, cB = 0.f;
  if (dp == nullptr) {
    // every wave forms the coefficients itself (no LDS hand-off, no barrier).  fpart: the
    // FocalTversky sums from the out_conv forward's partials in ftl_sums_kernel's order
    // (bit-identical to l3u_ftl_reduce; wave_sum_d leaves the same total in every lane)
    double sm[3];
    if (fpart != nullptr) {
      ftl_lane_sums(fpart, fnp, sm[0], sm[1], sm[2]);
    } else {
      sm[0] = sums[0]; sm[1] = sums[1]; sm[2] = sums[2];
    }
    const FtlCoef r = ftl_coef(sm, alpha, beta, gamma, smooth);
    const double s = gscale ? (double)gscale[0] : 1.0;
    cA = (float)(r.A * s);
    cB = (float)(r.B * s);
    if (loss && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) loss[0] = (float)r.loss;
  }
  f4 dz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (i0 + q < S) {
      const float pv = VEC ? pv4[q] : p[o + i0 + q];
      const float gs = VEC ? gv4[q] : (dp ? dp[o + i0 + q] : t[o + i0 + q]);
      const float g = dp ? gs : fmaf(cA - cB, gs, cB);
      dz[q] = g * pv * (1.f - pv);
    }
  }
  float acc[33];
#pragma unroll
  for (int c = 0; c < 33; ++c) acc[c] = 0.f;
  acc[32] = (dz[0] + dz[1]) + (dz[2] + dz[3]);
  if (dz_only) {   // d(pre-sigmoid) only: the consumers form dh[c] = w[c] * dz on the fly
    if (VEC) {
      if (i0 < S) stv4(dhp + i0, dz);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (i0 + q < S) st1(dhp + i0 + q, dz[q]);
    }
  }
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    if (c < C) {
      if (VEC) {
        if (i0 < S) {
          const f4 hc = hv[VEC ? c : 0];
          acc[c] = fmaf(dz[0], hc[0], fmaf(dz[1], hc[1], fmaf(dz[2], hc[2], dz[3] * hc[3])));
          if (!dz_only) stv4(dhp + (long long)c * S + i0, w[c] * dz);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (i0 + q < S) {
            acc[c] = fmaf(dz[q], ld1(hp + (long long)c * S + i0 + q), acc[c]);
            if (!dz_only) st1(dhp + (long long)c * S + i0 + q, w[c] * dz[q]);
          }
      }
    }
  }
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < 33; ++c) {
    if (c < C || c == 32) {
      const double r = wave_sum_d((double)acc[c]);
      if (l == 0) redd[wv * (C + 1) + (c == 32 ? C : c)] = r;
    }
  }
  __syncthreads();
  if (threadIdx.x <= C) {
    const int tt = threadIdx.x;
    const double r = (redd[tt] + redd[(C + 1) + tt]) + (redd[2 * (C + 1) + tt] + redd[3 * (C + 1) + tt]);
    part[((long long)n * nb + blockIdx.x) * (C + 1) + tt] = r;
  }
}

// ---------------------------------------------------------------- Focal-Tversky
// part[blk] = {sum p*t, sum p, sum t}
__global__ __launch_bounds__(256) void ftl_partials_kernel(const float* __restrict__ p,
                                                           const float* __restrict__ t,
                                                           long long numel,
                                                           float* __restrict__ part) {
  L3U_STAMP_SCOPE(405);
  __shared__ float red[4];
  float spt = 0.f, sp = 0.f, st = 0.f;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < numel; i += (long long)gridDim.x * 256) {
    const float pv = p[i], tv = t[i];
    spt = fmaf(pv, tv, spt);
    sp += pv;
    st += tv;
  }
  spt = block_sum256(spt, red);
  sp = block_sum256(sp, red);
  st = block_sum256(st, red);
  if (threadIdx.x == 0) {
    part[blockIdx.x * 3 + 0] = spt;
    part[blockIdx.x * 3 + 1] = sp;
    part[blockIdx.x * 3 + 2] = st;
  }
}

// sums[0..2] (double) = fixed-order sum of the partials
__global__ void ftl_sums_kernel(const float* __restrict__ part, int nb, double* __restrict__ sums) {
  L3U_STAMP_SCOPE(406);
  double a, b, c;
  ftl_lane_sums(part, nb, a, b, c);
  if (threadIdx.x == 0) { sums[0] = a; sums[1] = b; sums[2] = c; }
}

__global__ void ftl_loss_kernel(const double* __restrict__ sums, double alpha, double beta,
                                double gamma, double smooth, float* __restrict__ loss) {
  L3U_STAMP_SCOPE(407);
  const FtlCoef r = ftl_coef(sums, alpha, beta, gamma, smooth);
  loss[0] = (float)r.loss;
}

// g_i = gscale * (A t_i + B (1 - t_i)); optionally fused sigmoid backward: g_i *= p_i (1 - p_i)
__global__ __launch_bounds__(256) void ftl_bwd_kernel(
    const float* __restrict__ p, const float* __restrict__ t, long long numel,
    const double* __restrict__ sums, double alpha, double beta, double gamma, double smooth,
    const float* __restrict__ gscale, int through_sigmoid, float* __restrict__ g) {
  L3U_STAMP_SCOPE(408);
  __shared__ float coef[2];
  if (threadIdx.x == 0) {
    const FtlCoef r = ftl_coef(sums, alpha, beta, gamma, smooth);
    const double s = gscale ? (double)gscale[0] : 1.0;
    coef[0] = (float)(r.A * s);
    coef[1] = (float)(r.B * s);
  }
  __syncthreads();
  const float A = coef[0], B = coef[1];
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < numel; i += (long long)gridDim.x * 256) {
    const float tv = t[i];
    float v = fmaf(A - B, tv, B);
    if (through_sigmoid) { const float pv = p[i]; v *= pv * (1.f - pv); }
    g[i] = v;
  }
}

// ---------------------------------------------------------------- AdamW (torch.optim.AdamW)
// The per-element update, shared by adamw_tick and the fused reduce + update below so that both
// round identically.
struct AdamWStep { float step_size, decay, bc2s, beta1, beta2, eps, gscale; };
__device__ __forceinline__ AdamWStep adamw_step(float lrv, float beta1, float beta2, float eps,
                                                float wd, int t, float gscale) {
  AdamWStep c;
  const float bc1 = 1.f - powf(beta1, (float)t);
  c.bc2s = sqrtf(1.f - powf(beta2, (float)t));
  c.step_size = lrv / bc1;
  c.decay = 1.f - lrv * wd;
  c.beta1 = beta1; c.beta2 = beta2; c.eps = eps; c.gscale = gscale;
  return c;
}
__device__ __forceinline__ void adamw_update(const AdamWStep& c, float& pv, float gv, float& mv,
                                             float& vv) {
  // no FMA contraction: the rounding must not depend on how the surrounding kernel is scheduled
#pragma clang fp contract(off)
  gv *= c.gscale;
  pv *= c.decay;
  mv = mv + (1.f - c.beta1) * (gv - mv);                 // exp_avg.lerp_(grad, 1 - beta1)
  vv = vv * c.beta2 + (1.f - c.beta2) * gv * gv;
  const float denom = sqrtf(vv) / c.bc2s + c.eps;
  pv = pv - c.step_size * (mv / denom);
}

// One launch: the update, and the step counter(s) advanced by the LAST workgroup to finish (ticket
// order): every workgroup has read *step by the time it takes its ticket, so the increment
// cannot race a read, and the separate one-thread launch disappears.  The ticket is reset.
template <bool VEC>
__global__ __launch_bounds__(256) void adamw_tick_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         long long numel, const float* __restrict__ lr,
                                                         float beta1, float beta2, float eps, float wd,
                                                         int* step, float gscale, int* ticket,
                                                         int* counter2) {
  L3U_STAMP_SCOPE(409);
  const int t = step[0] + 1;
  const AdamWStep c = adamw_step(lr[0], beta1, beta2, eps, wd, t, gscale);
  auto upd = [&](float& pv, float gv, float& mv, float& vv) { adamw_update(c, pv, gv, mv, vv); };
  const long long st = (long long)gridDim.x * 256;
  if (VEC) {
    // float4 per thread: the four arrays' loads of a thread are one memory round trip (the scalar
    // grid-stride loop issued four dependent rounds); same per-element arithmetic
    const long long n4 = numel >> 2;
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += st) {
      f4 pv = ldv4(p + 4 * i), mv = ldv4(m + 4 * i), vv = ldv4(v + 4 * i);
      const f4 gv = ldv4(g + 4 * i);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float a = pv[q], b = mv[q], c = vv[q];
        upd(a, gv[q], b, c);
        pv[q] = a; mv[q] = b; vv[q] = c;
      }
      stv4(p + 4 * i, pv);
      stv4(m + 4 * i, mv);
      stv4(v + 4 * i, vv);
    }
    const long long i = 4 * n4 + threadIdx.x;
    if (blockIdx.x == 0 && i < numel) {
      float pv = p[i], mv = m[i], vv = v[i];
      upd(pv, g[i], mv, vv);
      p[i] = pv; m[i] = mv; v[i] = vv;
    }
  } else {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < numel; i += st) {
      float pv = p[i], mv = m[i], vv = v[i];
      upd(pv, g[i], mv, vv);
      p[i] = pv; m[i] = mv; v[i] = vv;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(ticket, 1) == (int)gridDim.x - 1) {
    step[0] = t;
    if (counter2) counter2[0] += 1;
    ticket[0] = 0;
  }
}

__global__ void counter_add_kernel(int* c, int v) { c[0] += v; }

// ---------------------------------------------------------------- segmented partial reduction
constexpr int kSegBatch = 8;   // measured: 8 < 16 < 32 us/step
#ifndef L3U_SEG_VEC
#define L3U_SEG_VEC 1
#endif
constexpr bool kSegVec = L3U_SEG_VEC != 0;   // float4 rows where the item allows (segment_sum)
#ifndef L3U_SEG_LONG
#define L3U_SEG_LONG 32
#endif
constexpr int kSegLong = L3U_SEG_LONG;   // terms per thread above which the scalar form doubles B
// item (8 x int64): src_off, count, istride, tstride, len, dst_off, accumulate, unused
// dst[dst_off + t] (+)= sum_{i<count} src[src_off + i*istride + t*tstride], t < len (<= 256)
// Returns, for thread t < len, the segment's sum for output t (red: 256 doubles of LDS).
__device__ __forceinline__ double segment_sum(const float* __restrict__ src,
                                              const long long* __restrict__ it, double* red) {
  const int t = threadIdx.x;
  const int len = (int)it[4];
  // fp32 partial rows with 16-byte aligned, contiguous outputs (the pointwise / ConvTranspose3d
  // weight-gradient partials): a thread sums 4 adjacent outputs from float4 loads, so the 864- /
  // 432-long partial lists of the 48^3 / 24^3 layers take a quarter of the dependent load rounds
  // of the scalar form below (same fixed order per output: i = k, k + TP, ...; deterministic)
  // The item's base address is workgroup-uniform (scalar registers) and every per-lane offset
  // within it fits 32 bits: one offset VGPR per load in flight instead of a 64-bit address
  const float* __restrict__ sb = src + it[0];
  const int cnt = (int)it[1];
  if (kSegVec && !it[7] && it[3] == 1 && (len & 3) == 0 && (it[2] & 3) == 0 && (it[0] & 3) == 0) {
    const int L4 = len >> 2, TP = 256 / L4;
    const int o4 = t % L4, k = t / L4;
    const int is4 = (int)(it[2] >> 2);
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    if (k < TP) {
      const f4* __restrict__ sf = reinterpret_cast<const f4*>(sb);
      constexpr int B = kSegBatch;
      // every batch's loads in flight at once, the tail too: clamped (always valid) addresses and
      // unconditional loads, the out-of-range terms dropped by a select AFTER the load (a
      // predicated load made the compiler branch around each load with a vmcnt(0) inside)
      for (int i = k; i < cnt; i += B * TP) {
        f4 v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) v[u] = sf[o4 + min(i + u * TP, cnt - 1) * is4];
#pragma unroll
        for (int u = 0; u < B; ++u) {
          const bool ok = i + u * TP < cnt;
#pragma unroll
          for (int q = 0; q < 4; ++q) s[q] += ok ? (double)v[u][q] : 0.0;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) red[t * 4 + q] = s[q];
    __syncthreads();
    double r = 0.0;
    if (t < len)
      for (int kk = 0; kk < TP; ++kk) r += red[(kk * L4 + (t >> 2)) * 4 + (t & 3)];
    return r;
  }
  // TP threads per output: thread (k, o) sums terms i = k, k+TP, k+2TP, ... of output o
  // (consecutive threads on consecutive outputs: coalesced), then the TP partial sums are added
  // in k order.  TP depends only on len, so the summation order is fixed: deterministic.  Lists
  // longer than kSegLong terms per thread (the one-channel 48^3 depthwise partials: 107 per
  // thread) keep twice the loads in flight (half the dependent rounds; same order of the adds)
  const int TP = 256 / len;
  const int o = t % len, k = t / len;
  const int is = (int)it[2], base = o * (int)it[3];
  double s = 0.0;
  auto sum = [&](auto BB) {
    constexpr int B = decltype(BB)::value;   // loads in flight per thread
    for (int i = k; i < cnt; i += B * TP) {
      float v[B];
#pragma unroll
      for (int u = 0; u < B; ++u) v[u] = sb[base + min(i + u * TP, cnt - 1) * is];
#pragma unroll
      for (int u = 0; u < B; ++u) s += i + u * TP < cnt ? (double)v[u] : 0.0;
    }
  };
  if (k < TP) {
    if (it[7]) {   // fp64 partials (src_off and strides count doubles; the lists are short)
      constexpr int B = kSegBatch;
      const double* __restrict__ sd = reinterpret_cast<const double*>(src) + it[0];
      for (int i = k; i < cnt; i += B * TP) {
        double v[B];
#pragma unroll
        for (int u = 0; u < B; ++u) v[u] = sd[base + min(i + u * TP, cnt - 1) * is];
#pragma unroll
        for (int u = 0; u < B; ++u) s += i + u * TP < cnt ? v[u] : 0.0;
      }
    } else if (cnt > kSegLong * TP) {
      sum(std::integral_constant<int, 2 * kSegBatch>{});
    } else {
      sum(std::integral_constant<int, kSegBatch>{});
    }
  }
  red[t] = s;
  __syncthreads();
  double r = 0.0;
  if (t < len)
    for (int kk = 0; kk < TP; ++kk) r += red[kk * len + t];
  return r;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void reduce_segments_kernel(const float* __restrict__ src,
                                                              const long long* __restrict__ items,
                                                              float* __restrict__ dst) {
  L3U_STAMP_SCOPE(410);
  __shared__ double red[1024];   // segment_sum: 4 per thread in the float4 form
  const long long* it = items + (long long)blockIdx.x * 8;
  const double r = segment_sum(src, it, red);
  const int t = threadIdx.x;
  if (t < (int)it[4]) {
    float* d = dst + it[5] + t;
    *d = it[6] ? (float)((double)*d + r) : (float)r;
  }
}

// One process, every parameter written by exactly one non-accumulating item: the segment's
// reduced gradient goes straight into the AdamW update of its parameters (the gradient is still
// stored).  The step counter(s) advance as in adamw_tick_kernel (ticket order).  The parameter /
// moment loads are issued before the reduction so their round trip overlaps it.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void reduce_segments_adamw_kernel(
    const float* __restrict__ src, const long long* __restrict__ items, float* __restrict__ g,
    float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
    const float* __restrict__ lr, float beta1, float beta2, float eps, float wd, int* step,
    float gscale, int* ticket, int* counter2) {
  L3U_STAMP_SCOPE(416);
  __shared__ double red[1024];   // segment_sum: 4 per thread in the float4 form
  const long long* it = items + (long long)blockIdx.x * 8;
  const int tc = step[0] + 1;
  const float lrv = lr[0];
  const int t = threadIdx.x;
  const bool mine = t < (int)it[4];
  const long long j = it[5] + t;
  float pv = 0.f, mv = 0.f, vv = 0.f;
  if (mine) { pv = p[j]; mv = m[j]; vv = v[j]; }
  const double r = segment_sum(src, it, red);
  if (mine) {
    const float gv = (float)r;
    g[j] = gv;
    adamw_update(adamw_step(lrv, beta1, beta2, eps, wd, tc, gscale), pv, gv, mv, vv);
    p[j] = pv; m[j] = mv; v[j] = vv;
  }
  __syncthreads();
  // two-level ticket: thousands of workgroups taking one device-scope atomic serialize on that
  // address (measured +16 us at 2.6k workgroups); L3U_TICKET_GROUPS counters a cache line apart
  // take a share each, and the last workgroup of each group takes the top ticket[0]
  if (threadIdx.x == 0) {
    constexpr int G = L3U_TICKET_GROUPS;
    const int nb = (int)gridDim.x, gr = (int)blockIdx.x % G, ng = nb < G ? nb : G;
    const int n_in = (nb - gr + G - 1) / G;
    int* tg = ticket + L3U_TICKET_STRIDE * (gr + 1);
    if (atomicAdd(tg, 1) == n_in - 1) {
      tg[0] = 0;
      if (atomicAdd(ticket, 1) == ng - 1) {
        step[0] = tc;
        if (counter2) counter2[0] += 1;
        ticket[0] = 0;
      }
    }
  }
}

// Vector forms for even D, H and W % 4 == 0 (every pooled level of the network): one thread per
// pair of x-adjacent outputs reads the 2x2 rows of its 2x2x4 input block as four float4 loads and
// writes the pair (float2) and its two argmax bytes; the backward writes the same block as four
// float4 stores.  Same scan order and comparison as the scalar kernels above.
template <typename T>
__global__ __launch_bounds__(256) void maxpool2_fwd_v_kernel(
    const T* __restrict__ x, long long xns, T* __restrict__ y, long long yns,
    unsigned char* __restrict__ idx, int C, int D, int H, int W) {
  L3U_STAMP_SCOPE(411);
  const int Ho = H / 2, W4 = W / 4;
  const long long So = (long long)(D / 2) * Ho * (W / 2), Si = (long long)D * H * W;
  const long long Sp = So / 2;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const T* xp = x + (long long)n * xns + (long long)c * Si;
  T* yp = y + (long long)n * yns + (long long)c * So;
  unsigned short* ip = reinterpret_cast<unsigned short*>(idx + (long long)nc * So);
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < Sp; o += (long long)gridDim.x * 256) {
    const int q = (int)(o % W4), t = (int)(o / W4), oy = t % Ho, oz = t / Ho;
    const T* b = xp + ((long long)(2 * oz) * H + 2 * oy) * W + 4 * q;
    f4 r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = ldv4(b + ((long long)(j >> 1) * H + (j & 1)) * W);
    float b0 = r[0][0], b1 = r[0][2];
    int i0 = 0, i1 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v0[2] = {r[j][0], r[j][1]}, v1[2] = {r[j][2], r[j][3]};
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        if (j == 0 && dx == 0) continue;
        if (v0[dx] > b0 || v0[dx] != v0[dx]) { b0 = v0[dx]; i0 = 2 * j + dx; }
        if (v1[dx] > b1 || v1[dx] != v1[dx]) { b1 = v1[dx]; i1 = 2 * j + dx; }
      }
    }
    stv2(yp + 2 * o, f2_t{b0, b1});
    ip[o] = (unsigned short)(i0 | (i1 << 8));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool2_bwd_v_kernel(
    const T* __restrict__ dy, long long dyns, const unsigned char* __restrict__ idx,
    const T* __restrict__ add, long long addns, T* __restrict__ dx, long long dxns,
    int C, int D, int H, int W) {
  L3U_STAMP_SCOPE(412);
  const int Ho = H / 2, W4 = W / 4;
  const long long So = (long long)(D / 2) * Ho * (W / 2), Si = (long long)D * H * W;
  const long long Sp = So / 2;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const T* dyp = dy + (long long)n * dyns + (long long)c * So;
  const unsigned short* ip = reinterpret_cast<const unsigned short*>(idx + (long long)nc * So);
  const T* ap = add ? add + (long long)n * addns + (long long)c * Si : nullptr;
  T* dxp = dx + (long long)n * dxns + (long long)c * Si;
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < Sp; o += (long long)gridDim.x * 256) {
    const int q = (int)(o % W4), t = (int)(o / W4), oy = t % Ho, oz = t / Ho;
    const long long base = ((long long)(2 * oz) * H + 2 * oy) * W + 4 * q;
    const f2_t g = ldv2(dyp + 2 * o);
    const int id = ip[o], i0 = id & 0xff, i1 = id >> 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long off = base + ((long long)(j >> 1) * H + (j & 1)) * W;
      f4 v = ap ? ldv4(ap + off) : f4{0.f, 0.f, 0.f, 0.f};
      v[0] += i0 == 2 * j ? g.x : 0.f;
      v[1] += i0 == 2 * j + 1 ? g.x : 0.f;
      v[2] += i1 == 2 * j ? g.y : 0.f;
      v[3] += i1 == 2 * j + 1 ? g.y : 0.f;
      stv4(dxp + off, v);
    }
  }
}

// the vector kernels need even D and H, W % 4 == 0 and 16-byte aligned channel planes
bool pool_vec_ok(int D, int H, int W, const void* a, long long ans, const void* b, long long bns,
                 const void* c, long long cns, int esize) {
  if ((D & 1) || (H & 1) || (W & 3)) return false;
  const void* p[3] = {a, b, c};
  const long long ns[3] = {ans, bns, cns};
  for (int i = 0; i < 3; ++i)
    if (p[i] && (((uintptr_t)p[i] & (4 * esize - 1)) || (ns[i] & 3))) return false;
  return true;
}

int grid_for(long long n, int per_block, int cap) {
  long long b = (n + per_block - 1) / per_block;
  if (b > cap) b = cap;
  return b < 1 ? 1 : (int)b;
}

// ---------------------------------------------------------------- first block front (Cin = 1)
// The first ResidualBlock of the network has ONE input channel (unet3d.py:163-167), so its
// Conv1x1 shortcut and conv1.pointwise are rank-1 "GEMMs": r[c] = wr[c] * x and y1[c] = w1[c] * z1
// with z1 = depthwise3(x) (conv1.depthwise, one channel).  One launch reads x once, writes z1
// (kept for the backward) and both C-channel tensors, and emits their InstanceNorm statistics
// partials, derived from the block's single-channel moments: a channel's (count, mean, M2) over
// the workgroup's voxels is (count, w*mean, w^2*M2) of the input channel, exactly.
// One workgroup per 1024 voxels (a float4 quad per thread) of one sample.
// xc != NULL: also a copy of x in the storage type (the bf16 network's backward reads x as bf16).
// y1 / r may be NULL (fp32): they are never materialised, their consumers form them on load.
template <typename T>
__global__ __launch_bounds__(256) void front_fwd_kernel(
    const float* __restrict__ x, long long xns, const float* __restrict__ wdw,
    const float* __restrict__ w1, const float* __restrict__ wr, T* __restrict__ z1,
    T* __restrict__ y1, T* __restrict__ r, float* __restrict__ stat1,
    float* __restrict__ statr, T* __restrict__ xc, int C, int D, int H, int W) {
  L3U_STAMP_SCOPE(413);
  __shared__ float red[4];
  const int S = D * H * W, nb = gridDim.x, b = blockIdx.x, n = blockIdx.y;
  const int i0 = (b * 256 + threadIdx.x) * 4;
  const bool act = i0 < S;
  const float* xp = x + (long long)n * xns;
  f4 xv = {0.f, 0.f, 0.f, 0.f}, zv = {0.f, 0.f, 0.f, 0.f};
  // every operand requested in one round trip: the 9 neighbourhood rows (float4 + the two edge
  // values) at clamped addresses without branches (a branch around each row's loads had the
  // compiler wait for the previous row first: nine dependent round trips), rows outside the
  // volume zeroed after the load; the taps (scalar loads) beside them.  Same fma order and
  // values as before: a zeroed row adds +0 to the accumulator that started at +0.
  const int ic = act ? i0 : 0;
  const int xx = ic % W, t1 = ic / W, yy = t1 % H, zz = t1 / H;   // quad: xx .. xx+3, one row
  f4 m9[9];
  float l9[9], r9[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int zr = min(max(zz + k / 3 - 1, 0), D - 1), yr = min(max(yy + k % 3 - 1, 0), H - 1);
    const float* row = xp + ((long long)zr * H + yr) * W;
    m9[k] = *reinterpret_cast<const f4*>(row + xx);
    l9[k] = row[max(xx - 1, 0)];
    r9[k] = row[min(xx + 4, W - 1)];
  }
  xv = m9[4];
  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = wdw[t];
  if (act) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int dz = k / 3 - 1, dy = k % 3 - 1;
      const bool in = zz + dz >= 0 && zz + dz < D && yy + dy >= 0 && yy + dy < H;
      const f4 m = in ? m9[k] : f4{0.f, 0.f, 0.f, 0.f};
      const float lft = in && xx > 0 ? l9[k] : 0.f, rgt = in && xx + 4 < W ? r9[k] : 0.f;
      const float v[6] = {lft, m[0], m[1], m[2], m[3], rgt};
      const float* w3 = wk + k * 3;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        zv[q] = fmaf(w3[0], v[q], fmaf(w3[1], v[q + 1], fmaf(w3[2], v[q + 2], zv[q])));
    }
    stv4(z1 + (long long)n * S + i0, zv);
    if (xc) stv4(xc + (long long)n * S + i0, xv);
    // r / y1 == NULL: the consumers take them rank-1 (wr[c] * x, w1[c] * z1; include/l3u.h)
    if (r != nullptr)
      for (int c = 0; c < C; ++c) stv4(r + ((long long)n * C + c) * S + i0, wr[c] * xv);
    if (y1 != nullptr)
      for (int c = 0; c < C; ++c) stv4(y1 + ((long long)n * C + c) * S + i0, w1[c] * zv);
  }
  // the workgroup's moments of x and z1 (fixed-order sums: deterministic)
  const int cnt = min(1024, S - b * 1024);
  const float sx = block_sum256(act ? (xv[0] + xv[1]) + (xv[2] + xv[3]) : 0.f, red);
  const float sz = block_sum256(act ? (zv[0] + zv[1]) + (zv[2] + zv[3]) : 0.f, red);
  const float mx = sx / (float)cnt, mz = sz / (float)cnt;
  float qx = 0.f, qz = 0.f;
  if (act) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      qx = fmaf(xv[q] - mx, xv[q] - mx, qx);
      qz = fmaf(zv[q] - mz, zv[q] - mz, qz);
    }
  }
  const float m2x = block_sum256(qx, red), m2z = block_sum256(qz, red);
  for (int c = threadIdx.x; c < C; c += 256) {
    float* o1 = stat1 + (((long long)n * C + c) * nb + b) * 3;
    float* orr = statr + (((long long)n * C + c) * nb + b) * 3;
    o1[0] = (float)cnt; o1[1] = w1[c] * mz; o1[2] = w1[c] * w1[c] * m2z;
    orr[0] = (float)cnt; orr[1] = wr[c] * mx; orr[2] = wr[c] * wr[c] * m2x;
  }
}

// ---------------------------------------------------------------- pad / crop (UpBlock)
// dst[n][c][z][y][x] = src[n][c][z - oz][y - oy][x - ox] where that lies inside src's box, else 0:
// F.pad of the ConvTranspose3d output to the skip volume (oz, oy, ox >= 0, unet3d.py:130-138) and,
// with the offsets negated, its backward (the crop of the concat gradient).  One thread per dst
// voxel, x fastest: the stores are contiguous rows, the loads contiguous runs of src rows.
template <typename T>
__global__ __launch_bounds__(256) void box_copy_kernel(
    const T* __restrict__ src, long long sns, int sd, int sh, int sw, T* __restrict__ dst,
    long long dns, int dd, int dh, int dw, int oz, int oy, int ox, int C, long long total) {
  L3U_STAMP_SCOPE(414);
  const long long dS = (long long)dd * dh * dw, sS = (long long)sd * sh * sw;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int x = (int)(i % dw);
    long long t = i / dw;
    const int y = (int)(t % dh);
    t /= dh;
    const int z = (int)(t % dd);
    t /= dd;
    const int c = (int)(t % C), n = (int)(t / C);
    const int zs = z - oz, ys = y - oy, xs = x - ox;
    float v = 0.f;
    if (zs >= 0 && zs < sd && ys >= 0 && ys < sh && xs >= 0 && xs < sw)
      v = ld1(src + n * sns + c * sS + ((long long)zs * sh + ys) * sw + xs);
    st1(dst + n * dns + c * dS + ((long long)z * dh + y) * dw + x, v);
  }
}

// ---------------------------------------------------------------- storage casts
template <typename S_, typename D_>
__global__ __launch_bounds__(256) void cast_kernel(const S_* __restrict__ x, D_* __restrict__ y,
                                                   long long n4, long long n) {
  L3U_STAMP_SCOPE(415);
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256)
    stv4(y + 4 * i, ldv4(x + 4 * i));
  const long long t = 4 * n4 + blockIdx.x * 256ll + threadIdx.x;
  if (blockIdx.x == 0 && t < n) st1(y + t, ld1(x + t));
}

template <typename T>
int maxpool2_fwd_impl(const T* x, long long x_nstride, T* y, long long y_nstride,
                      unsigned char* idx, int N, int C, int D, int H, int W, hipStream_t stream) {
  constexpr int E = (int)sizeof(T);
  L3U_REQUIRE(N > 0 && C > 0 && D >= 2 && H >= 2 && W >= 2);
  const long long So = (long long)(D / 2) * (H / 2) * (W / 2);
  if (pool_vec_ok(D, H, W, x, x_nstride, nullptr, 0, nullptr, 0, E) &&
      ((uintptr_t)y & (2 * E - 1)) == 0 && (y_nstride & 1) == 0 && ((uintptr_t)idx & 1) == 0)
    hipLaunchKernelGGL(maxpool2_fwd_v_kernel<T>, dim3(grid_for(So / 2, 256, 64), N * C), dim3(256), 0,
                       stream, x, x_nstride, y, y_nstride, idx, C, D, H, W);
  else
    hipLaunchKernelGGL(maxpool2_fwd_kernel<T>, dim3(grid_for(So, 256, 64), N * C), dim3(256), 0,
                       stream, x, x_nstride, y, y_nstride, idx, C, D, H, W);
  L3U_CHECK_LAUNCH();
}

template <typename T>
int maxpool2_bwd_impl(const T* dy, long long dy_nstride, const unsigned char* idx, const T* add,
                      long long add_nstride, T* dx, long long dx_nstride, int N, int C, int D,
                      int H, int W, hipStream_t stream) {
  constexpr int E = (int)sizeof(T);
  L3U_REQUIRE(N > 0 && C > 0 && D >= 2 && H >= 2 && W >= 2);
  const long long Si = (long long)D * H * W;
  if (pool_vec_ok(D, H, W, add, add_nstride, dx, dx_nstride, nullptr, 0, E) &&
      ((uintptr_t)dy & (2 * E - 1)) == 0 && (dy_nstride & 1) == 0 && ((uintptr_t)idx & 1) == 0)
    hipLaunchKernelGGL(maxpool2_bwd_v_kernel<T>, dim3(grid_for(Si / 16, 256, 64), N * C), dim3(256),
                       0, stream, dy, dy_nstride, idx, add, add_nstride, dx, dx_nstride, C, D, H, W);
  else
    hipLaunchKernelGGL(maxpool2_bwd_kernel<T>, dim3(grid_for(Si, 256, 128), N * C), dim3(256), 0,
                       stream, dy, dy_nstride, idx, add, add_nstride, dx, dx_nstride, C, D, H, W);
  L3U_CHECK_LAUNCH();
}

template <typename T>
int outconv_fwd_impl(const T* h, long long h_nstride, const float* w, const float* b, float* p,
                     const float* t, float* ftl_part, int N, int C, int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0);
  L3U_REQUIRE(t == nullptr || ftl_part != nullptr);
  const bool vec = S % 4 == 0 && h_nstride % 4 == 0 && C <= 32;   // the vector form holds <= 32 channels
  dim3 grid((S + 1023) / 1024, N);
  if (vec) hipLaunchKernelGGL((outconv_fwd_kernel<T, true>), grid, dim3(256), 0, stream, h, h_nstride, w, b, p, t, ftl_part, C, S);
  else hipLaunchKernelGGL((outconv_fwd_kernel<T, false>), grid, dim3(256), 0, stream, h, h_nstride, w, b, p, t, ftl_part, C, S);
  L3U_CHECK_LAUNCH();
}

template <typename T>
int outconv_bwd_impl(const float* dp, const float* p, const float* t, const double* sums,
                     double alpha, double beta, double gamma, double smooth, const float* gscale,
                     const T* h, long long h_nstride, const float* w, float* dh, long long dh_nstride,
                     double* part, float* loss, int N, int C, int S, hipStream_t stream,
                     const float* fpart = nullptr, int fnp = 0, int dz_only = 0) {
  L3U_REQUIRE(N > 0 && C > 0 && C <= 32 && S > 0);
  L3U_REQUIRE(dp != nullptr || (t != nullptr && (sums != nullptr || (fpart != nullptr && fnp > 0))));
  const bool vec = S % 4 == 0 && h_nstride % 4 == 0 && dh_nstride % 4 == 0;
  dim3 grid((S + 1023) / 1024, N);
  const size_t lds = 4 * (C + 1) * sizeof(double);
  if (vec) hipLaunchKernelGGL((outconv_bwd_kernel<T, true>), grid, dim3(256), lds, stream, dz_only, dp, p, t, sums, alpha, beta, gamma, smooth, gscale, h, h_nstride, w, dh, dh_nstride, part, loss, C, S, fpart, fnp);
  else hipLaunchKernelGGL((outconv_bwd_kernel<T, false>), grid, dim3(256), lds, stream, dz_only, dp, p, t, sums, alpha, beta, gamma, smooth, gscale, h, h_nstride, w, dh, dh_nstride, part, loss, C, S, fpart, fnp);
  L3U_CHECK_LAUNCH();
}

template <typename T>
int front_fwd_impl(const float* x, long long x_nstride, const float* w_dw, const float* w1,
                   const float* wr, T* z1, T* y1, T* r, float* stat1, float* statr, T* xc, int N,
                   int C, int D, int H, int W, hipStream_t stream) {
  constexpr int E = (int)sizeof(T);
  L3U_REQUIRE(N > 0 && C > 0 && D > 0 && H > 0 && W > 0 && W % 4 == 0 && x_nstride % 4 == 0);
  L3U_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)z1 & (4 * E - 1)) == 0 &&
              ((uintptr_t)y1 & (4 * E - 1)) == 0 && ((uintptr_t)r & (4 * E - 1)) == 0 &&
              ((uintptr_t)xc & (4 * E - 1)) == 0);
  const int S = D * H * W;
  dim3 grid((S + 1023) / 1024, N);
  hipLaunchKernelGGL(front_fwd_kernel<T>, grid, dim3(256), 0, stream, x, x_nstride, w_dw, w1, wr, z1,
                     y1, r, stat1, statr, xc, C, D, H, W);
  L3U_CHECK_LAUNCH();
}

}  // namespace

#define P_MPF(TT) (const TT* x, long long x_nstride, TT* y, long long y_nstride, unsigned char* idx, \
    int N, int C, int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_maxpool2_fwd, P_MPF, maxpool2_fwd_impl(bp(x), x_nstride, bp(y), y_nstride, idx, N, C, D,
         H, W, stream))
extern "C" int l3u_maxpool2_bwd(const float* dy, long long dy_nstride, const unsigned char* idx,
                                const float* add, long long add_nstride, float* dx,
                                long long dx_nstride, int N, int C, int D, int H, int W,
                                hipStream_t stream) {
  return maxpool2_bwd_impl(dy, dy_nstride, idx, add, add_nstride, dx, dx_nstride, N, C, D, H, W,
                           stream);
}
#define P_OCF(TT) (const TT* h, long long h_nstride, const float* w, const float* b, float* p,        \
    const float* t, float* ftl_part, int N, int C, int S, hipStream_t stream)
L3U_TWIN(l3u_outconv_fwd, P_OCF, outconv_fwd_impl(bp(h), h_nstride, w, b, p, t, ftl_part, N, C, S,
         stream))
#define P_OCB(TT) (const float* dp, const float* p, const float* t, const double* sums, double alpha, \
    double beta, double gamma, double smooth, const float* gscale, const TT* h, long long h_nstride, \
    const float* w, float* dh, long long dh_nstride, double* part, float* loss, int N, int C, int S, \
    hipStream_t stream)
L3U_TWIN(l3u_outconv_bwd, P_OCB, outconv_bwd_impl(dp, p, t, sums, alpha, beta, gamma, smooth, gscale,
         bp(h), h_nstride, w, dh, dh_nstride, part, loss, N, C, S, stream))
#define P_OCBF(TT) (const float* p, const float* t, const float* ftl_part, int ftl_nparts,           \
    double alpha, double beta, double gamma, double smooth, const float* gscale, const TT* h,         \
    long long h_nstride, const float* w, float* dh, long long dh_nstride, double* part, float* loss,  \
    int N, int C, int S, hipStream_t stream)
L3U_TWIN(l3u_outconv_bwd_ftl, P_OCBF, outconv_bwd_impl((const float*)nullptr, p, t, (const double*)nullptr,
         alpha, beta, gamma, smooth, gscale, bp(h), h_nstride, w, dh, dh_nstride, part, loss, N, C, S,
         stream, ftl_part, ftl_nparts))
// the same two forms writing dz = d(pre-sigmoid) [N][S] (batch stride dz_nstride) instead of dh:
// out_conv is rank-1 (dh[c] = w[c] * dz), so the last block's tail consumers read dz (the _r1
// entry points) and dh is never stored
L3U_TWIN(l3u_outconv_bwd_dz, P_OCB, outconv_bwd_impl(dp, p, t, sums, alpha, beta, gamma, smooth, gscale,
         bp(h), h_nstride, w, dh, dh_nstride, part, loss, N, C, S, stream, nullptr, 0, 1))
L3U_TWIN(l3u_outconv_bwd_ftl_dz, P_OCBF, outconv_bwd_impl((const float*)nullptr, p, t,
         (const double*)nullptr, alpha, beta, gamma, smooth, gscale, bp(h), h_nstride, w, dh, dh_nstride,
         part, loss, N, C, S, stream, ftl_part, ftl_nparts, 1))
template <typename T>
int box_copy_impl(const T* src, long long sns, int sd, int sh, int sw, T* dst, long long dns, int dd,
                  int dh, int dw, int oz, int oy, int ox, int N, int C, hipStream_t stream) {
  L3U_REQUIRE(src && dst && N > 0 && C > 0 && sd > 0 && sh > 0 && sw > 0 && dd > 0 && dh > 0 && dw > 0);
  const long long total = (long long)N * C * dd * dh * dw;
  hipLaunchKernelGGL((box_copy_kernel<T>), dim3(grid_for(total, 256, 8192)), dim3(256), 0, stream, src,
                     sns, sd, sh, sw, dst, dns, dd, dh, dw, oz, oy, ox, C, total);
  L3U_CHECK_LAUNCH();
}
#define P_BOX(TT) (const TT* src, long long src_nstride, int sd, int sh, int sw, TT* dst,            \
    long long dst_nstride, int dd, int dh, int dw, int oz, int oy, int ox, int N, int C,             \
    hipStream_t stream)
L3U_TWIN(l3u_box_copy, P_BOX, box_copy_impl(bp(src), src_nstride, sd, sh, sw, bp(dst), dst_nstride, dd,
         dh, dw, oz, oy, ox, N, C, stream))
#define P_FRF(TT) (const float* x, long long x_nstride, const float* w_dw, const float* w1,          \
    const float* wr, TT* z1, TT* y1, TT* r, float* stat1, float* statr, TT* x_copy, int N, int C,    \
    int D, int H, int W, hipStream_t stream)
L3U_TWIN(l3u_front_fwd, P_FRF, front_fwd_impl(x, x_nstride, w_dw, w1, wr, bp(z1), bp(y1), bp(r), stat1,
         statr, bp(x_copy), N, C, D, H, W, stream))

extern "C" {

int l3u_cast_f32_bf16(const float* x, l3u_bf16* y, long long n, hipStream_t stream) {
  L3U_REQUIRE(n > 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 7) == 0);
  hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(grid_for(n / 4 + 1, 256, 1024)), dim3(256), 0,
                     stream, x, bp(y), n / 4, n);
  L3U_CHECK_LAUNCH();
}

int l3u_cast_bf16_f32(const l3u_bf16* x, float* y, long long n, hipStream_t stream) {
  L3U_REQUIRE(n > 0 && ((uintptr_t)x & 7) == 0 && ((uintptr_t)y & 15) == 0);
  hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(grid_for(n / 4 + 1, 256, 1024)), dim3(256), 0,
                     stream, bp(x), y, n / 4, n);
  L3U_CHECK_LAUNCH();
}


int l3u_outconv_nblocks(int S) { return (S + 1023) / 1024; }

int l3u_ftl_reduce(const float* part, int nparts, double* sums, hipStream_t stream) {
  L3U_REQUIRE(nparts > 0);
  hipLaunchKernelGGL(ftl_sums_kernel, dim3(1), dim3(64), 0, stream, part, nparts, sums);
  L3U_CHECK_LAUNCH();
}

int l3u_ftl_nblocks(long long numel) { return grid_for(numel, 2048, 512); }

int l3u_ftl_sums(const float* p, const float* t, long long numel, float* part, double* sums,
                 hipStream_t stream) {
  L3U_REQUIRE(numel > 0);
  const int nb = grid_for(numel, 2048, 512);
  hipLaunchKernelGGL(ftl_partials_kernel, dim3(nb), dim3(256), 0, stream, p, t, numel, part);
  hipLaunchKernelGGL(ftl_sums_kernel, dim3(1), dim3(64), 0, stream, part, nb, sums);
  L3U_CHECK_LAUNCH();
}

int l3u_ftl_loss(const double* sums, double alpha, double beta, double gamma, double smooth,
                 float* loss, hipStream_t stream) {
  hipLaunchKernelGGL(ftl_loss_kernel, dim3(1), dim3(1), 0, stream, sums, alpha, beta, gamma, smooth,
                     loss);
  L3U_CHECK_LAUNCH();
}

int l3u_ftl_bwd(const float* p, const float* t, long long numel, const double* sums, double alpha,
                double beta, double gamma, double smooth, const float* gscale,
                int through_sigmoid, float* g, hipStream_t stream) {
  L3U_REQUIRE(numel > 0);
  hipLaunchKernelGGL(ftl_bwd_kernel, dim3(grid_for(numel, 1024, 1024)), dim3(256), 0, stream, p, t,
                     numel, sums, alpha, beta, gamma, smooth, gscale, through_sigmoid, g);
  L3U_CHECK_LAUNCH();
}

int l3u_front_nblocks(int S) { return (S + 1023) / 1024; }

int l3u_adamw_tick(float* p, const float* g, float* m, float* v, long long numel, const float* lr,
                   float beta1, float beta2, float eps, float weight_decay, int* step,
                   float grad_scale, int* ticket, int* counter2, hipStream_t stream) {
  L3U_REQUIRE(numel > 0 && step && ticket);
  const bool vec = ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0;
  if (vec)
    hipLaunchKernelGGL(adamw_tick_kernel<true>, dim3(grid_for(numel, 1024, 1024)), dim3(256), 0, stream,
                       p, g, m, v, numel, lr, beta1, beta2, eps, weight_decay, step, grad_scale, ticket,
                       counter2);
  else
    hipLaunchKernelGGL(adamw_tick_kernel<false>, dim3(grid_for(numel, 1024, 1024)), dim3(256), 0, stream,
                       p, g, m, v, numel, lr, beta1, beta2, eps, weight_decay, step, grad_scale, ticket,
                       counter2);
  L3U_CHECK_LAUNCH();
}

int l3u_reduce_segments(const float* src, const long long* items, int nitems, float* dst,
                        hipStream_t stream) {
  // src 16-byte aligned: segment_sum's float4 rows check only the item's own offset (it[0] % 4)
  L3U_REQUIRE(nitems > 0 && src && ((uintptr_t)src & 15) == 0);
  hipLaunchKernelGGL(reduce_segments_kernel, dim3(nitems), dim3(256), 0, stream, src, items, dst);
  L3U_CHECK_LAUNCH();
}

int l3u_reduce_segments_adamw(const float* src, const long long* items, int nitems, float* g,
                              float* p, float* m, float* v, const float* lr, float beta1,
                              float beta2, float eps, float weight_decay, int* step,
                              float grad_scale, int* ticket, int* counter2, hipStream_t stream) {
  L3U_REQUIRE(nitems > 0 && step && ticket && src && ((uintptr_t)src & 15) == 0);
  hipLaunchKernelGGL(reduce_segments_adamw_kernel, dim3(nitems), dim3(256), 0, stream, src, items,
                     g, p, m, v, lr, beta1, beta2, eps, weight_decay, step, grad_scale, ticket,
                     counter2);
  L3U_CHECK_LAUNCH();
}

int l3u_counter_add(int* counter, int value, hipStream_t stream) {
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, stream, counter, value);
  L3U_CHECK_LAUNCH();
}

int l3u_abi_version(void) { return L3U_ABI_VERSION; }

}  // extern "C"

#ifdef L3U_STAMP
// Wave-stamp registry of the profiling variant build (common.h StampScope): every translation
// unit registers the setter of its own device pointers; l3u_stamp_setup installs one buffer in
// all of them (buf: cap StampRec records, ctr: 256 zeroed unsigned; NULL buf turns stamping off).
namespace l3u {
static std::vector<void (*)(void*, void*, unsigned)>& stamp_setters() {
  static std::vector<void (*)(void*, void*, unsigned)> v;
  return v;
}
void stamp_register(void (*set)(void*, void*, unsigned)) { stamp_setters().push_back(set); }
}  // namespace l3u
extern "C" int l3u_stamp_setup(void* buf, void* ctr, unsigned cap) {
  for (auto f : l3u::stamp_setters()) f(buf, ctr, cap);
  return (int)hipDeviceSynchronize();
}
#endif
