// Remaining hot-path ops:
//   maxpool2_fwd/bwd     nn.MaxPool3d(2, 2)                                   unet3d.py:101
//   convt_d2s / s2d      the scatter half of nn.ConvTranspose3d(k=2, s=2)     unet3d.py:119,127
//                        (the GEMM half is l3u_pw_fwd with Nout = Co*8)
//   chan_sum             per-channel sums (bias gradients)
//   outconv fwd/bwd      out_conv 1x1x1 (+bias) + Sigmoid                      unet3d.py:201-202,220-221
//   ftl_*                FocalTverskyLoss forward sums / loss / closed-form backward  losses.py:30-54
//   adamw                torch.optim.AdamW step on the flat parameter buffer     trainer.py:75-79
//   reduce_segments      deterministic second stage of every split-K / partial reduction
#include "common.h"
using namespace l3u;

typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

// ---------------------------------------------------------------- maxpool 2x2x2 (floor mode)
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(
    const float* __restrict__ x, long long xns, float* __restrict__ y, long long yns,
    unsigned char* __restrict__ idx, int C, int D, int H, int W) {
  const int Do = D / 2, Ho = H / 2, Wo = W / 2;
  const long long So = (long long)Do * Ho * Wo, Si = (long long)D * H * W;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const float* xp = x + (long long)n * xns + (long long)c * Si;
  float* yp = y + (long long)n * yns + (long long)c * So;
  unsigned char* ip = idx + (long long)nc * So;
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < So; o += (long long)gridDim.x * 256) {
    const int ox = (int)(o % Wo), t = (int)(o / Wo), oy = t % Ho, oz = t / Ho;
    const float* b = xp + ((long long)(2 * oz) * H + 2 * oy) * W + 2 * ox;
    float best = b[0];
    int bi = 0;
    // scan order (dz, dy, dx) and strict '>' (first maximum wins; NaN propagates) as torch CPU
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      const int dz = j >> 2, dy = (j >> 1) & 1, dx = j & 1;
      const float v = b[((long long)dz * H + dy) * W + dx];
      if (v > best || v != v) { best = v; bi = j; }
    }
    yp[o] = best;
    ip[o] = (unsigned char)bi;
  }
}

// dx = route(dy) (+ add): every input voxel is written exactly once (covers odd-size tails)
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(
    const float* __restrict__ dy, long long dyns, const unsigned char* __restrict__ idx,
    const float* __restrict__ add, long long addns, float* __restrict__ dx, long long dxns,
    int C, int D, int H, int W) {
  const int Do = D / 2, Ho = H / 2, Wo = W / 2;
  const long long So = (long long)Do * Ho * Wo, Si = (long long)D * H * W;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const float* dyp = dy + (long long)n * dyns + (long long)c * So;
  const unsigned char* ip = idx + (long long)nc * So;
  const float* ap = add ? add + (long long)n * addns + (long long)c * Si : nullptr;
  float* dxp = dx + (long long)n * dxns + (long long)c * Si;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < Si; i += (long long)gridDim.x * 256) {
    const int xx = (int)(i % W), t = (int)(i / W), yy = t % H, zz = t / H;
    float v = 0.f;
    const int oz = zz >> 1, oy = yy >> 1, ox = xx >> 1;
    if (oz < Do && oy < Ho && ox < Wo) {
      const long long o = ((long long)oz * Ho + oy) * Wo + ox;
      const int j = ((zz & 1) << 2) | ((yy & 1) << 1) | (xx & 1);
      if (ip[o] == j) v = dyp[o];
    }
    if (ap) v += ap[i];
    dxp[i] = v;
  }
}

// ---------------------------------------------------------------- ConvTranspose3d(k2,s2) scatter
// Yp[n][co*8 + a*4 + b*2 + c][z][y][x] (+bias[co]) -> out[n][co][2z+a][2y+b][2x+c]
__global__ __launch_bounds__(256) void convt_d2s_kernel(
    const float* __restrict__ yp, const float* __restrict__ bias, float* __restrict__ out,
    long long ons, int Co, int D, int H, int W) {
  const int D2 = 2 * D, H2 = 2 * H, W2 = 2 * W;
  const long long So = (long long)D2 * H2 * W2, Si = (long long)D * H * W;
  const int nc = blockIdx.y, co = nc % Co, n = nc / Co;
  const float bv = bias ? bias[co] : 0.f;
  const float* src = yp + ((long long)n * Co * 8 + (long long)co * 8) * Si;
  float* dst = out + (long long)n * ons + (long long)co * So;
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < So; o += (long long)gridDim.x * 256) {
    const int X = (int)(o % W2), t = (int)(o / W2), Y = t % H2, Z = t / H2;
    const int par = ((Z & 1) << 2) | ((Y & 1) << 1) | (X & 1);
    dst[o] = src[par * Si + ((long long)(Z >> 1) * H + (Y >> 1)) * W + (X >> 1)] + bv;
  }
}

// dYp[n][co*8+par][s_in] = dy[n][co][...]
__global__ __launch_bounds__(256) void convt_s2d_kernel(
    const float* __restrict__ dy, long long dyns, float* __restrict__ dyp, int Co, int D, int H,
    int W) {
  const int D2 = 2 * D, H2 = 2 * H, W2 = 2 * W;
  const long long So = (long long)D2 * H2 * W2, Si = (long long)D * H * W;
  const int nc = blockIdx.y, co = nc % Co, n = nc / Co;
  const float* src = dy + (long long)n * dyns + (long long)co * So;
  float* dst = dyp + ((long long)n * Co * 8 + (long long)co * 8) * Si;
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < So; o += (long long)gridDim.x * 256) {
    const int X = (int)(o % W2), t = (int)(o / W2), Y = t % H2, Z = t / H2;
    const int par = ((Z & 1) << 2) | ((Y & 1) << 1) | (X & 1);
    dst[par * Si + ((long long)(Z >> 1) * H + (Y >> 1)) * W + (X >> 1)] = src[o];
  }
}

// ---------------------------------------------------------------- per-channel sums
// part[c][n][blk] = sum over the block's voxel range of x[n][c][:]
__global__ __launch_bounds__(256) void chan_sum_kernel(const float* __restrict__ x, long long xns,
                                                       double* __restrict__ part, int N, int C,
                                                       long long S) {
  __shared__ double red[4];
  const int nc = blockIdx.y, c = nc % C, n = nc / C, nb = gridDim.x;
  const float* xp = x + (long long)n * xns + (long long)c * S;
  double s = 0.0;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < S; i += (long long)nb * 256) s += xp[i];
  s = block_sum256d(s, red);
  if (threadIdx.x == 0) part[((long long)c * N + n) * nb + blockIdx.x] = s;
}

// ---------------------------------------------------------------- out_conv + sigmoid
// p = sigmoid(b + sum_c w[c] h[c]); 4 voxels per thread (float4 when VEC).  t != NULL: also the
// FocalTversky partials of this block, ftl_part[n*nb + blk] = {sum p*t, sum p, sum t} (the loss's
// first reduction stage fused into the producer of p: losses.py:40-42).
template <bool VEC>
__global__ __launch_bounds__(256) void outconv_fwd_kernel(
    const float* __restrict__ h, long long hns, const float* __restrict__ w,
    const float* __restrict__ b, float* __restrict__ p, const float* __restrict__ t,
    float* __restrict__ ftl_part, int C, int S) {
  __shared__ float red[4];
  const int n = blockIdx.y;
  const float* hp = h + (long long)n * hns;
  float* pp = p + (long long)n * S;
  const float bv = b[0];
  const int i0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  f4 z = {bv, bv, bv, bv};
  if (VEC) {
    if (i0 < S) {
      for (int c = 0; c < C; ++c) z += w[c] * *reinterpret_cast<const f4*>(hp + (long long)c * S + i0);
    }
  } else {
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (i0 + q < S) z[q] = fmaf(w[c], hp[(long long)c * S + i0 + q], z[q]);
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
      const float tv = t[(long long)n * S + i0 + q];
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
// TAIL: also the first stage of the last decoder block's tail backward (l3u_norm_act_bwd_reduce
// of up3, whose output IS h): tpart[c][n][nb][3] = {sum g, sum g*xhat2, sum g*xhat_r} over the
// workgroup's voxels, g = dh * lrelu'(h), so dh and h are not read again for it.
template <bool VEC, bool TAIL = false>
__global__ __launch_bounds__(256) void outconv_bwd_kernel(
    const float* __restrict__ dp, const float* __restrict__ p, const float* __restrict__ t,
    const double* __restrict__ sums, double alpha, double beta, double gamma, double smooth,
    const float* __restrict__ gscale, const float* __restrict__ h, long long hns,
    const float* __restrict__ w, float* __restrict__ dh, long long dhns,
    double* __restrict__ part, float* __restrict__ loss, int C, int S,
    const float* __restrict__ y2 = nullptr, long long y2ns = 0, const float* __restrict__ rec2 = nullptr,
    const float* __restrict__ r = nullptr, long long rns = 0, const float* __restrict__ recr = nullptr,
    double* __restrict__ tpart = nullptr, int N = 0) {
  extern __shared__ double redd[];   // [4][C+1] (TAIL: [4][3C])
  __shared__ float coef[2];
  const int n = blockIdx.y, nb = gridDim.x;
  if (dp == nullptr) {
    if (threadIdx.x == 0) {
      const FtlCoef r = ftl_coef(sums, alpha, beta, gamma, smooth);
      const double s = gscale ? (double)gscale[0] : 1.0;
      coef[0] = (float)(r.A * s);
      coef[1] = (float)(r.B * s);
      if (loss && blockIdx.x == 0 && blockIdx.y == 0) loss[0] = (float)r.loss;
    }
    __syncthreads();
  }
  const float* hp = h + (long long)n * hns;
  float* dhp = dh + (long long)n * dhns;
  const long long o = (long long)n * S;
  const int i0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  f4 dz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (i0 + q < S) {
      const float pv = p[o + i0 + q];
      const float g = dp ? dp[o + i0 + q] : fmaf(coef[0] - coef[1], t[o + i0 + q], coef[1]);
      dz[q] = g * pv * (1.f - pv);
    }
  }
  float acc[33];
#pragma unroll
  for (int c = 0; c < 33; ++c) acc[c] = 0.f;
  acc[32] = (dz[0] + dz[1]) + (dz[2] + dz[3]);
  float ts[TAIL ? 3 * 16 : 1];
  if (TAIL) {
#pragma unroll
    for (int c = 0; c < 3 * 16; ++c) ts[c] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    if (c < C) {
      if (VEC) {
        if (i0 < S) {
          const f4 hv = *reinterpret_cast<const f4*>(hp + (long long)c * S + i0);
          acc[c] = fmaf(dz[0], hv[0], fmaf(dz[1], hv[1], fmaf(dz[2], hv[2], dz[3] * hv[3])));
          const f4 dhv = w[c] * dz;
          *reinterpret_cast<f4*>(dhp + (long long)c * S + i0) = dhv;
          if (TAIL && c < 16) {   // same float expressions as norm_act_bwd_reduce_kernel
            const float* q2 = rec2 + ((long long)n * C + c) * kRec;
            const float* qr = recr + ((long long)n * C + c) * kRec;
            const float m2 = q2[0], rs2 = q2[1], mr = qr[0], rsr = qr[1];
            const f4 yv = *reinterpret_cast<const f4*>(y2 + (long long)n * y2ns + (long long)c * S + i0);
            const f4 rv = *reinterpret_cast<const f4*>(r + (long long)n * rns + (long long)c * S + i0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float g = dhv[q] * lrelu_d(hv[q]);
              ts[3 * c] += g;
              ts[3 * c + 1] += g * ((yv[q] - m2) * rs2);
              ts[3 * c + 2] += g * ((rv[q] - mr) * rsr);
            }
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (i0 + q < S) {
            acc[c] = fmaf(dz[q], hp[(long long)c * S + i0 + q], acc[c]);
            dhp[(long long)c * S + i0 + q] = w[c] * dz[q];
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
  if (TAIL) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 3 * 16; ++e) {
      if (e < 3 * C) {
        const double v = wave_sum_d((double)ts[e]);
        if (l == 0) redd[wv * 3 * C + e] = v;
      }
    }
    __syncthreads();
    if (threadIdx.x < 3 * C) {
      const int e = threadIdx.x, c = e / 3, k = e - 3 * c;
      const double v = (redd[e] + redd[3 * C + e]) + (redd[6 * C + e] + redd[9 * C + e]);
      tpart[(((long long)c * N + n) * nb + blockIdx.x) * 3 + k] = v;
    }
  }
}

// ---------------------------------------------------------------- Focal-Tversky
// part[blk] = {sum p*t, sum p, sum t}
__global__ __launch_bounds__(256) void ftl_partials_kernel(const float* __restrict__ p,
                                                           const float* __restrict__ t,
                                                           long long numel,
                                                           float* __restrict__ part) {
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
  __shared__ double red[3][64];
  const int l = threadIdx.x;   // 64 threads
  double a = 0, b = 0, c = 0;
  for (int i = l; i < nb; i += 64) { a += part[i * 3]; b += part[i * 3 + 1]; c += part[i * 3 + 2]; }
  red[0][l] = a; red[1][l] = b; red[2][l] = c;
  __syncthreads();
  if (l < 3) {
    double s = 0;
    for (int i = 0; i < 64; ++i) s += red[l][i];
    sums[l] = s;
  }
}

__global__ void ftl_loss_kernel(const double* __restrict__ sums, double alpha, double beta,
                                double gamma, double smooth, float* __restrict__ loss) {
  const FtlCoef r = ftl_coef(sums, alpha, beta, gamma, smooth);
  loss[0] = (float)r.loss;
}

// g_i = gscale * (A t_i + B (1 - t_i)); optionally fused sigmoid backward: g_i *= p_i (1 - p_i)
__global__ __launch_bounds__(256) void ftl_bwd_kernel(
    const float* __restrict__ p, const float* __restrict__ t, long long numel,
    const double* __restrict__ sums, double alpha, double beta, double gamma, double smooth,
    const float* __restrict__ gscale, int through_sigmoid, float* __restrict__ g) {
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
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    long long numel, const float* __restrict__ lr,
                                                    float beta1, float beta2, float eps, float wd,
                                                    const int* __restrict__ step, float gscale) {
  const float lrv = lr[0];
  const int t = step[0] + 1;
  const float bc1 = 1.f - powf(beta1, (float)t);
  const float bc2s = sqrtf(1.f - powf(beta2, (float)t));
  const float step_size = lrv / bc1;
  const float decay = 1.f - lrv * wd;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < numel; i += (long long)gridDim.x * 256) {
    const float gv = g[i] * gscale;
    float pv = p[i] * decay;
    float mv = m[i];
    mv = mv + (1.f - beta1) * (gv - mv);                 // exp_avg.lerp_(grad, 1 - beta1)
    const float vv = v[i] * beta2 + (1.f - beta2) * gv * gv;
    const float denom = sqrtf(vv) / bc2s + eps;
    pv = pv - step_size * (mv / denom);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
}

// The same update with the step counter(s) advanced by the LAST workgroup to finish (ticket
// order): every workgroup has read *step by the time it takes its ticket, so the increment
// cannot race a read, and the separate one-thread launch disappears.  The ticket is reset.
__global__ __launch_bounds__(256) void adamw_tick_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         long long numel, const float* __restrict__ lr,
                                                         float beta1, float beta2, float eps, float wd,
                                                         int* step, float gscale, int* ticket,
                                                         int* counter2) {
  const float lrv = lr[0];
  const int t = step[0] + 1;
  const float bc1 = 1.f - powf(beta1, (float)t);
  const float bc2s = sqrtf(1.f - powf(beta2, (float)t));
  const float step_size = lrv / bc1;
  const float decay = 1.f - lrv * wd;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < numel; i += (long long)gridDim.x * 256) {
    const float gv = g[i] * gscale;
    float pv = p[i] * decay;
    float mv = m[i];
    mv = mv + (1.f - beta1) * (gv - mv);                 // exp_avg.lerp_(grad, 1 - beta1)
    const float vv = v[i] * beta2 + (1.f - beta2) * gv * gv;
    const float denom = sqrtf(vv) / bc2s + eps;
    pv = pv - step_size * (mv / denom);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(ticket, 1) == (int)gridDim.x - 1) {
    step[0] = t;
    if (counter2) counter2[0] += 1;
    ticket[0] = 0;
  }
}

__global__ void step_inc_kernel(int* step) { step[0] += 1; }
__global__ void counter_add_kernel(int* c, int v) { c[0] += v; }

// ---------------------------------------------------------------- segmented partial reduction
// item (8 x int64): src_off, count, istride, tstride, len, dst_off, accumulate, unused
// dst[dst_off + t] (+)= sum_{i<count} src[src_off + i*istride + t*tstride], t < len (<= 256)
__global__ __launch_bounds__(256) void reduce_segments_kernel(const float* __restrict__ src,
                                                              const long long* __restrict__ items,
                                                              float* __restrict__ dst) {
  __shared__ double red[256];
  const long long* it = items + (long long)blockIdx.x * 8;
  const int t = threadIdx.x;
  const int len = (int)it[4];
  // TP threads per output: thread (k, o) sums terms i = k, k+TP, k+2TP, ... of output o
  // (consecutive threads on consecutive outputs: coalesced), then the TP partial sums are added
  // in k order.  TP depends only on len, so the summation order is fixed: deterministic.
  const int TP = 256 / len;
  const int o = t % len, k = t / len;
  const long long cnt = it[1], is = it[2];
  double s = 0.0;
  if (k < TP) {
    const long long base = it[0] + o * it[3];
    const long long stp = is * TP;
    long long i = k;
    if (it[7]) {
      const double* sd = reinterpret_cast<const double*>(src) + base;
      for (; i + 15 * TP < cnt; i += 16 * TP) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = sd[i * is + u * stp];
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
      }
      for (; i < cnt; i += TP) s += sd[i * is];
    } else {
      const float* sf = src + base;
      for (; i + 15 * TP < cnt; i += 16 * TP) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = sf[i * is + u * stp];
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
      }
      for (; i < cnt; i += TP) s += sf[i * is];
    }
  }
  red[t] = s;
  __syncthreads();
  if (t < len) {
    double r = 0.0;
    for (int kk = 0; kk < TP; ++kk) r += red[kk * len + t];
    float* d = dst + it[5] + t;
    *d = it[6] ? (float)((double)*d + r) : (float)r;
  }
}

// Vector forms for even D, H and W % 4 == 0 (every pooled level of the network): one thread per
// pair of x-adjacent outputs reads the 2x2 rows of its 2x2x4 input block as four float4 loads and
// writes the pair (float2) and its two argmax bytes; the backward writes the same block as four
// float4 stores.  Same scan order and comparison as the scalar kernels above.
__global__ __launch_bounds__(256) void maxpool2_fwd_v_kernel(
    const float* __restrict__ x, long long xns, float* __restrict__ y, long long yns,
    unsigned char* __restrict__ idx, int C, int D, int H, int W) {
  const int Ho = H / 2, W4 = W / 4;
  const long long So = (long long)(D / 2) * Ho * (W / 2), Si = (long long)D * H * W;
  const long long Sp = So / 2;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const float* xp = x + (long long)n * xns + (long long)c * Si;
  float2* yp = reinterpret_cast<float2*>(y + (long long)n * yns + (long long)c * So);
  unsigned short* ip = reinterpret_cast<unsigned short*>(idx + (long long)nc * So);
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < Sp; o += (long long)gridDim.x * 256) {
    const int q = (int)(o % W4), t = (int)(o / W4), oy = t % Ho, oz = t / Ho;
    const float* b = xp + ((long long)(2 * oz) * H + 2 * oy) * W + 4 * q;
    float4 r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      r[j] = *reinterpret_cast<const float4*>(b + ((long long)(j >> 1) * H + (j & 1)) * W);
    float b0 = r[0].x, b1 = r[0].z;
    int i0 = 0, i1 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float v0[2] = {r[j].x, r[j].y}, v1[2] = {r[j].z, r[j].w};
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        if (j == 0 && dx == 0) continue;
        if (v0[dx] > b0 || v0[dx] != v0[dx]) { b0 = v0[dx]; i0 = 2 * j + dx; }
        if (v1[dx] > b1 || v1[dx] != v1[dx]) { b1 = v1[dx]; i1 = 2 * j + dx; }
      }
    }
    yp[o] = make_float2(b0, b1);
    ip[o] = (unsigned short)(i0 | (i1 << 8));
  }
}

__global__ __launch_bounds__(256) void maxpool2_bwd_v_kernel(
    const float* __restrict__ dy, long long dyns, const unsigned char* __restrict__ idx,
    const float* __restrict__ add, long long addns, float* __restrict__ dx, long long dxns,
    int C, int D, int H, int W) {
  const int Ho = H / 2, W4 = W / 4;
  const long long So = (long long)(D / 2) * Ho * (W / 2), Si = (long long)D * H * W;
  const long long Sp = So / 2;
  const int nc = blockIdx.y, c = nc % C, n = nc / C;
  const float2* dyp = reinterpret_cast<const float2*>(dy + (long long)n * dyns + (long long)c * So);
  const unsigned short* ip = reinterpret_cast<const unsigned short*>(idx + (long long)nc * So);
  const float* ap = add ? add + (long long)n * addns + (long long)c * Si : nullptr;
  float* dxp = dx + (long long)n * dxns + (long long)c * Si;
  for (long long o = blockIdx.x * 256ll + threadIdx.x; o < Sp; o += (long long)gridDim.x * 256) {
    const int q = (int)(o % W4), t = (int)(o / W4), oy = t % Ho, oz = t / Ho;
    const long long base = ((long long)(2 * oz) * H + 2 * oy) * W + 4 * q;
    const float2 g = dyp[o];
    const int id = ip[o], i0 = id & 0xff, i1 = id >> 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long off = base + ((long long)(j >> 1) * H + (j & 1)) * W;
      float4 v = ap ? *reinterpret_cast<const float4*>(ap + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      v.x += i0 == 2 * j ? g.x : 0.f;
      v.y += i0 == 2 * j + 1 ? g.x : 0.f;
      v.z += i1 == 2 * j ? g.y : 0.f;
      v.w += i1 == 2 * j + 1 ? g.y : 0.f;
      *reinterpret_cast<float4*>(dxp + off) = v;
    }
  }
}

// the vector kernels need even D and H, W % 4 == 0 and 16-byte aligned channel planes
bool pool_vec_ok(int D, int H, int W, const void* a, long long ans, const void* b, long long bns,
                 const void* c, long long cns) {
  if ((D & 1) || (H & 1) || (W & 3)) return false;
  const void* p[3] = {a, b, c};
  const long long ns[3] = {ans, bns, cns};
  for (int i = 0; i < 3; ++i)
    if (p[i] && (((uintptr_t)p[i] & 15) || (ns[i] & 3))) return false;
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
__global__ __launch_bounds__(256) void front_fwd_kernel(
    const float* __restrict__ x, long long xns, const float* __restrict__ wdw,
    const float* __restrict__ w1, const float* __restrict__ wr, float* __restrict__ z1,
    float* __restrict__ y1, float* __restrict__ r, float* __restrict__ stat1,
    float* __restrict__ statr, int C, int D, int H, int W) {
  __shared__ float red[4];
  const int S = D * H * W, nb = gridDim.x, b = blockIdx.x, n = blockIdx.y;
  const int i0 = (b * 256 + threadIdx.x) * 4;
  const bool act = i0 < S;
  const float* xp = x + (long long)n * xns;
  f4 xv = {0.f, 0.f, 0.f, 0.f}, zv = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    xv = *reinterpret_cast<const f4*>(xp + i0);
    const int xx = i0 % W, t1 = i0 / W, yy = t1 % H, zz = t1 / H;   // quad: xx .. xx+3, one row
#pragma unroll
    for (int dz = -1; dz <= 1; ++dz) {
      if (zz + dz < 0 || zz + dz >= D) continue;
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy) {
        if (yy + dy < 0 || yy + dy >= H) continue;
        const float* row = xp + ((long long)(zz + dz) * H + (yy + dy)) * W;
        const f4 m = *reinterpret_cast<const f4*>(row + xx);
        const float lft = xx > 0 ? row[xx - 1] : 0.f, rgt = xx + 4 < W ? row[xx + 4] : 0.f;
        const float v[6] = {lft, m[0], m[1], m[2], m[3], rgt};
        const float* wk = wdw + ((dz + 1) * 3 + (dy + 1)) * 3;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          zv[q] = fmaf(wk[0], v[q], fmaf(wk[1], v[q + 1], fmaf(wk[2], v[q + 2], zv[q])));
      }
    }
    *reinterpret_cast<f4*>(z1 + (long long)n * S + i0) = zv;
    for (int c = 0; c < C; ++c) {
      *reinterpret_cast<f4*>(r + ((long long)n * C + c) * S + i0) = wr[c] * xv;
      *reinterpret_cast<f4*>(y1 + ((long long)n * C + c) * S + i0) = w1[c] * zv;
    }
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

}  // namespace

extern "C" {

int l3u_maxpool2_fwd(const float* x, long long x_nstride, float* y, long long y_nstride,
                     unsigned char* idx, int N, int C, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && D >= 2 && H >= 2 && W >= 2);
  const long long So = (long long)(D / 2) * (H / 2) * (W / 2);
  if (pool_vec_ok(D, H, W, x, x_nstride, nullptr, 0, nullptr, 0) && ((uintptr_t)y & 7) == 0 &&
      (y_nstride & 1) == 0 && ((uintptr_t)idx & 1) == 0)
    hipLaunchKernelGGL(maxpool2_fwd_v_kernel, dim3(grid_for(So / 2, 256, 64), N * C), dim3(256), 0,
                       stream, x, x_nstride, y, y_nstride, idx, C, D, H, W);
  else
    hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(grid_for(So, 256, 64), N * C), dim3(256), 0, stream,
                       x, x_nstride, y, y_nstride, idx, C, D, H, W);
  L3U_CHECK_LAUNCH();
}

int l3u_maxpool2_bwd(const float* dy, long long dy_nstride, const unsigned char* idx,
                     const float* add, long long add_nstride, float* dx, long long dx_nstride,
                     int N, int C, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && D >= 2 && H >= 2 && W >= 2);
  const long long Si = (long long)D * H * W;
  if (pool_vec_ok(D, H, W, add, add_nstride, dx, dx_nstride, nullptr, 0) &&
      ((uintptr_t)dy & 7) == 0 && (dy_nstride & 1) == 0 && ((uintptr_t)idx & 1) == 0)
    hipLaunchKernelGGL(maxpool2_bwd_v_kernel, dim3(grid_for(Si / 16, 256, 64), N * C), dim3(256), 0,
                       stream, dy, dy_nstride, idx, add, add_nstride, dx, dx_nstride, C, D, H, W);
  else
    hipLaunchKernelGGL(maxpool2_bwd_kernel, dim3(grid_for(Si, 256, 128), N * C), dim3(256), 0, stream,
                       dy, dy_nstride, idx, add, add_nstride, dx, dx_nstride, C, D, H, W);
  L3U_CHECK_LAUNCH();
}

int l3u_convt_d2s(const float* yp, const float* bias, float* out, long long out_nstride, int N,
                  int Co, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && Co > 0 && D > 0 && H > 0 && W > 0);
  const long long So = 8ll * D * H * W;
  hipLaunchKernelGGL(convt_d2s_kernel, dim3(grid_for(So, 256, 128), N * Co), dim3(256), 0, stream,
                     yp, bias, out, out_nstride, Co, D, H, W);
  L3U_CHECK_LAUNCH();
}

int l3u_convt_s2d(const float* dy, long long dy_nstride, float* dyp, int N, int Co, int D, int H,
                  int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && Co > 0 && D > 0 && H > 0 && W > 0);
  const long long So = 8ll * D * H * W;
  hipLaunchKernelGGL(convt_s2d_kernel, dim3(grid_for(So, 256, 128), N * Co), dim3(256), 0, stream,
                     dy, dy_nstride, dyp, Co, D, H, W);
  L3U_CHECK_LAUNCH();
}

int l3u_chan_sum_nblocks(long long S) { return grid_for(S, 1024, 64); }

int l3u_chan_sum(const float* x, long long x_nstride, double* part, int N, int C, long long S,
                 hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0);
  hipLaunchKernelGGL(chan_sum_kernel, dim3(grid_for(S, 1024, 64), N * C), dim3(256), 0, stream, x,
                     x_nstride, part, N, C, S);
  L3U_CHECK_LAUNCH();
}

int l3u_outconv_nblocks(int S) { return (S + 1023) / 1024; }

int l3u_outconv_fwd(const float* h, long long h_nstride, const float* w, const float* b, float* p,
                    const float* t, float* ftl_part, int N, int C, int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && S > 0);
  L3U_REQUIRE(t == nullptr || ftl_part != nullptr);
  const bool vec = S % 4 == 0 && h_nstride % 4 == 0;
  dim3 grid((S + 1023) / 1024, N);
  if (vec) hipLaunchKernelGGL(outconv_fwd_kernel<true>, grid, dim3(256), 0, stream, h, h_nstride, w, b, p, t, ftl_part, C, S);
  else hipLaunchKernelGGL(outconv_fwd_kernel<false>, grid, dim3(256), 0, stream, h, h_nstride, w, b, p, t, ftl_part, C, S);
  L3U_CHECK_LAUNCH();
}

int l3u_outconv_bwd(const float* dp, const float* p, const float* t, const double* sums, double alpha,
                    double beta, double gamma, double smooth, const float* gscale, const float* h,
                    long long h_nstride, const float* w, float* dh, long long dh_nstride,
                    double* part, float* loss, int N, int C, int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && C <= 32 && S > 0);
  L3U_REQUIRE(dp != nullptr || (t != nullptr && sums != nullptr));
  const bool vec = S % 4 == 0 && h_nstride % 4 == 0 && dh_nstride % 4 == 0;
  dim3 grid((S + 1023) / 1024, N);
  const size_t lds = 4 * (C + 1) * sizeof(double);
  if (vec) hipLaunchKernelGGL((outconv_bwd_kernel<true, false>), grid, dim3(256), lds, stream, dp, p, t, sums, alpha, beta, gamma, smooth, gscale, h, h_nstride, w, dh, dh_nstride, part, loss, C, S);
  else hipLaunchKernelGGL((outconv_bwd_kernel<false, false>), grid, dim3(256), lds, stream, dp, p, t, sums, alpha, beta, gamma, smooth, gscale, h, h_nstride, w, dh, dh_nstride, part, loss, C, S);
  L3U_CHECK_LAUNCH();
}

int l3u_outconv_bwd_tail(const float* dp, const float* p, const float* t, const double* sums,
                         double alpha, double beta, double gamma, double smooth,
                         const float* gscale, const float* h, long long h_nstride, const float* w,
                         float* dh, long long dh_nstride, double* part, float* loss,
                         const float* y2, long long y2_nstride, const float* rec2, const float* r,
                         long long r_nstride, const float* rec_r, double* tail_part, int N, int C,
                         int S, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && C <= 16 && S > 0 && S % 4 == 0);
  L3U_REQUIRE(dp != nullptr || (t != nullptr && sums != nullptr));
  L3U_REQUIRE(y2 && rec2 && r && rec_r && tail_part);
  L3U_REQUIRE(h_nstride % 4 == 0 && dh_nstride % 4 == 0 && y2_nstride % 4 == 0 && r_nstride % 4 == 0);
  dim3 grid((S + 1023) / 1024, N);
  const size_t lds = 4 * 3 * (C + 1) * sizeof(double);
  hipLaunchKernelGGL((outconv_bwd_kernel<true, true>), grid, dim3(256), lds, stream, dp, p, t, sums,
                     alpha, beta, gamma, smooth, gscale, h, h_nstride, w, dh, dh_nstride, part, loss,
                     C, S, y2, y2_nstride, rec2, r, r_nstride, rec_r, tail_part, N);
  L3U_CHECK_LAUNCH();
}

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

int l3u_adamw(float* p, const float* g, float* m, float* v, long long numel, const float* lr,
              float beta1, float beta2, float eps, float weight_decay, int* step, float grad_scale,
              hipStream_t stream) {
  L3U_REQUIRE(numel > 0);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(numel, 1024, 1024)), dim3(256), 0, stream, p, g, m,
                     v, numel, lr, beta1, beta2, eps, weight_decay, step, grad_scale);
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, stream, step);
  L3U_CHECK_LAUNCH();
}

int l3u_front_nblocks(int S) { return (S + 1023) / 1024; }

int l3u_front_fwd(const float* x, long long x_nstride, const float* w_dw, const float* w1,
                  const float* wr, float* z1, float* y1, float* r, float* stat1, float* statr,
                  int N, int C, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && D > 0 && H > 0 && W > 0 && W % 4 == 0 && x_nstride % 4 == 0);
  L3U_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)z1 & 15) == 0 && ((uintptr_t)y1 & 15) == 0 &&
              ((uintptr_t)r & 15) == 0);
  const int S = D * H * W;
  dim3 grid(l3u_front_nblocks(S), N);
  hipLaunchKernelGGL(front_fwd_kernel, grid, dim3(256), 0, stream, x, x_nstride, w_dw, w1, wr, z1,
                     y1, r, stat1, statr, C, D, H, W);
  L3U_CHECK_LAUNCH();
}

int l3u_adamw_tick(float* p, const float* g, float* m, float* v, long long numel, const float* lr,
                   float beta1, float beta2, float eps, float weight_decay, int* step,
                   float grad_scale, int* ticket, int* counter2, hipStream_t stream) {
  L3U_REQUIRE(numel > 0 && step && ticket);
  hipLaunchKernelGGL(adamw_tick_kernel, dim3(grid_for(numel, 1024, 1024)), dim3(256), 0, stream, p, g,
                     m, v, numel, lr, beta1, beta2, eps, weight_decay, step, grad_scale, ticket,
                     counter2);
  L3U_CHECK_LAUNCH();
}

int l3u_reduce_segments(const float* src, const long long* items, int nitems, float* dst,
                        hipStream_t stream) {
  L3U_REQUIRE(nitems > 0);
  hipLaunchKernelGGL(reduce_segments_kernel, dim3(nitems), dim3(256), 0, stream, src, items, dst);
  L3U_CHECK_LAUNCH();
}

int l3u_counter_add(int* counter, int value, hipStream_t stream) {
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, stream, counter, value);
  L3U_CHECK_LAUNCH();
}

int l3u_abi_version(void) { return 1; }

}  // extern "C"
