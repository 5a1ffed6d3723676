// Depthwise 3x3x3 convolution (stride 1, zero padding 1, no bias) — forward and fused backward.
// Replaces nn.Conv3d(C, C, 3, 1, 1, groups=C, bias=False)   light_unet/models/unet3d.py:16-17.
//
// Mapping: one 256-thread workgroup owns one (n, c) channel volume and a slab of
// TZ output z-planes.  It walks the input planes z0-1 .. z0+TZ once ("2.5D" blocking): each plane
// is loaded coalesced (W contiguous) into a zero-haloed (H+2)x(W+2) LDS image, and each thread
// applies the 3 kernel slices of its (y, x) positions to 3 rolling register accumulators, so
// every input element is read from HBM once per slab and from LDS 9 times.  Next-plane global
// loads are issued before the current plane's stencil (register prefetch) so HBM latency hides
// under LDS/VALU work.  Logical workgroup ids are XCD-remapped so that slabs of one channel that
// share halo planes run on the same XCD (shared L2).
//
// MODE 1 fuses the InstanceNorm-apply + LeakyReLU + Dropout3d transform of the previous layer
// (unet3d.py:84-88) into the input load: a = lrelu(scale*y + shift), with zero padding applied in
// the transformed domain (as the reference pads the conv input a).
#include "common.h"
using namespace l3u;

namespace {

template <int MODE, int P>
__global__ __launch_bounds__(256) void dw3_fwd_kernel(
    const float* __restrict__ x, long long xns, const float* __restrict__ w,
    const float* __restrict__ rec, float* __restrict__ y, long long yns,
    int C, int D, int H, int W, int TZ, int nchunk) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int HW = H * W, PW = W + 2, PP = (H + 2) * PW;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = lb % nchunk;
  const int nc = lb / nchunk;
  const int c = nc % C, n = nc / C;
  const int z0 = chunk * TZ, z1 = min(z0 + TZ, D);
  const float* xp = x + (long long)n * xns + (long long)c * D * HW;
  float* yp = y + (long long)n * yns + (long long)c * D * HW;
  const int tid = threadIdx.x;

  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = w[c * 27 + t];
  float sc = 1.f, sh = 0.f, mu = 0.f;
  if (MODE == 1) {
    mu = rec[(long long)nc * kRec + 0];
    sc = rec[(long long)nc * kRec + 2];
    sh = rec[(long long)nc * kRec + 3];
  }
  for (int i = tid; i < 2 * PP; i += 256) lds[i] = 0.f;

  int lbase[P];
  bool own[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int p = tid + k * 256;
    own[k] = p < HW;
    const int yy = p / W, xx = p - yy * W;
    lbase[k] = own[k] ? (yy + 1) * PW + xx + 1 : 0;
  }
  float a0[P], a1[P], a2[P], nxt[P];
#pragma unroll
  for (int k = 0; k < P; ++k) { a0[k] = a1[k] = a2[k] = 0.f; nxt[k] = 0.f; }

  // prologue: fetch plane z0-1
  {
    const int zi = z0 - 1;
    if (zi >= 0) {
#pragma unroll
      for (int k = 0; k < P; ++k)
        if (own[k]) nxt[k] = xp[(long long)zi * HW + tid + k * 256];
    }
  }
  __syncthreads();
  for (int zi = z0 - 1; zi <= z1; ++zi) {
    float* buf = lds + ((zi - z0 + 1) & 1) * PP;
    const bool in = zi >= 0 && zi < D;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (own[k]) {
        float v = nxt[k];
        if (MODE == 1) v = lrelu(fmaf(sc, v - mu, sh));
        buf[lbase[k]] = in ? v : 0.f;
      }
    }
    // prefetch the next plane while this one is consumed
    const int zn = zi + 1;
    if (zn <= z1 && zn < D) {
#pragma unroll
      for (int k = 0; k < P; ++k)
        if (own[k]) nxt[k] = xp[(long long)zn * HW + tid + k * 256];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (!own[k]) continue;
      const float* b = buf + lbase[k];
      float v[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) v[dy * 3 + dx] = b[(dy - 1) * PW + (dx - 1)];
      // input plane zi feeds output plane zi+1 with slice kd=0, zi with kd=1, zi-1 with kd=2
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        a2[k] = fmaf(wk[j], v[j], a2[k]);
        a1[k] = fmaf(wk[9 + j], v[j], a1[k]);
        a0[k] = fmaf(wk[18 + j], v[j], a0[k]);
      }
    }
    const int zo = zi - 1;
    if (zo >= z0 && zo < z1) {
#pragma unroll
      for (int k = 0; k < P; ++k)
        if (own[k]) yp[(long long)zo * HW + tid + k * 256] = a0[k];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) { a0[k] = a1[k]; a1[k] = a2[k]; a2[k] = 0.f; }
  }
}

// Fused backward: dA = conv^T(dZ) (data gradient, flipped stencil) and dW = sum dZ (x) A (27 taps)
// in ONE pass over dZ and A.  Step s loads dZ plane zd = z0-1+s and A plane za = zd-1; the thread
// keeps its own dZ values of planes zd-2..zd in registers so each A-neighbourhood read from LDS
// feeds all three kernel depths.  dW is owned by the dZ plane (zd in [z0, z1)), so every product
// is counted exactly once across slabs.  Partial dW per workgroup -> dw_part[c][n*nchunk+chunk][27]
// (deterministic second stage: l3u_reduce_segments).
// MODE 1: A = lrelu(scale*y + shift) recomputed from y; the kernel emits
// dpre = dA * k * lrelu'(pre) (gradient at the InstanceNorm output before the activation) and the
// per-(n,c) partial sums  sum(dpre), sum(dpre * xhat)  for the InstanceNorm backward.
template <int MODE, int P>
__global__ __launch_bounds__(256) void dw3_bwd_kernel(
    const float* __restrict__ dz, long long dzns, const float* __restrict__ x, long long xns,
    const float* __restrict__ w, const float* __restrict__ rec, float* __restrict__ dx,
    long long dxns, int accumulate, float* __restrict__ dw_part, double* __restrict__ in_part,
    int N, int C, int D, int H, int W, int TZ, int nchunk) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int HW = H * W, PW = W + 2, PP = (H + 2) * PW;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = lb % nchunk;
  const int nc = lb / nchunk;
  const int c = nc % C, n = nc / C;
  const int z0 = chunk * TZ, z1 = min(z0 + TZ, D);
  const long long cofs = (long long)c * D * HW;
  const float* dzp = dz + (long long)n * dzns + cofs;
  const float* xp = x + (long long)n * xns + cofs;
  float* dxp = dx + (long long)n * dxns + cofs;
  const int tid = threadIdx.x;
  float* dzb = lds;            // 2 planes
  float* ab = lds + 2 * PP;    // 2 planes

  float wk[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) wk[t] = w[c * 27 + t];
  float sc = 1.f, sh = 0.f, kk = 1.f, mean = 0.f, rstd = 1.f;
  if (MODE == 1) {
    const float* r = rec + (long long)nc * kRec;
    mean = r[0]; rstd = r[1]; sc = r[2]; sh = r[3]; kk = r[4];
  }
  for (int i = tid; i < 4 * PP; i += 256) lds[i] = 0.f;

  int lbase[P];
  bool own[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int p = tid + k * 256;
    own[k] = p < HW;
    const int yy = p / W, xx = p - yy * W;
    lbase[k] = own[k] ? (yy + 1) * PW + xx + 1 : 0;
  }
  float d0[P], d1[P], d2[P];       // dA rolling accumulators for planes zd-1, zd, zd+1
  float g0[P], g1[P], g2[P];       // own dZ of planes zd-2, zd-1, zd (zero when not owned)
#pragma unroll
  for (int k = 0; k < P; ++k) d0[k] = d1[k] = d2[k] = g0[k] = g1[k] = g2[k] = 0.f;
  float gw[27];
#pragma unroll
  for (int t = 0; t < 27; ++t) gw[t] = 0.f;
  double s1 = 0.0, s2 = 0.0;

  const int zlo = max(0, z0 - 1), zhi = min(D - 1, z1);   // planes that carry data
  const int nsteps = z1 - z0 + 3;
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int zd = z0 - 1 + s, za = zd - 1;
    float* dbuf = dzb + (s & 1) * PP;
    float* abuf = ab + (s & 1) * PP;
    const bool ldz = zd >= zlo && zd <= zhi;
    const bool la = za >= zlo && za <= zhi;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (own[k]) {
        const long long off = tid + k * 256;
        dbuf[lbase[k]] = ldz ? dzp[(long long)zd * HW + off] : 0.f;
        float v = 0.f;
        if (la) {
          v = xp[(long long)za * HW + off];
          if (MODE == 1) v = lrelu(fmaf(sc, v - mean, sh));
        }
        abuf[lbase[k]] = v;
      }
    }
    __syncthreads();
    const bool zd_owned = zd >= z0 && zd < z1;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (!own[k]) continue;
      // dA: flipped stencil of dZ plane zd into dA planes zd-1 (kd=0), zd (kd=1), zd+1 (kd=2)
      const float* b = dbuf + lbase[k];
      float v[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dxx = 0; dxx < 3; ++dxx) v[dy * 3 + dxx] = b[(dy - 1) * PW + (dxx - 1)];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        d0[k] = fmaf(wk[8 - j], v[j], d0[k]);
        d1[k] = fmaf(wk[17 - j], v[j], d1[k]);
        d2[k] = fmaf(wk[26 - j], v[j], d2[k]);
      }
      g0[k] = g1[k];
      g1[k] = g2[k];
      g2[k] = zd_owned ? v[4] : 0.f;
      // dW: A plane za pairs with dZ planes za+1 (kd=0 -> g2), za (kd=1 -> g1), za-1 (kd=2 -> g0)
      const float* a = abuf + lbase[k];
      float u[9];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dxx = 0; dxx < 3; ++dxx) u[dy * 3 + dxx] = a[(dy - 1) * PW + (dxx - 1)];
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        gw[j] = fmaf(g2[k], u[j], gw[j]);
        gw[9 + j] = fmaf(g1[k], u[j], gw[9 + j]);
        gw[18 + j] = fmaf(g0[k], u[j], gw[18 + j]);
      }
    }
    const int zf = zd - 1;   // dA plane zf is complete
    if (zf >= z0 && zf < z1) {
#pragma unroll
      for (int k = 0; k < P; ++k) {
        if (!own[k]) continue;
        const long long idx = (long long)zf * HW + tid + k * 256;
        if (MODE == 1) {
          const float yv = xp[idx];
          const float pre = fmaf(sc, yv - mean, sh);
          const float dp = d0[k] * kk * lrelu_d(pre);
          const float xh = (yv - mean) * rstd;
          dxp[idx] = dp;
          s1 += dp;
          s2 += (double)dp * xh;
        } else {
          dxp[idx] = accumulate ? dxp[idx] + d0[k] : d0[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < P; ++k) { d0[k] = d1[k]; d1[k] = d2[k]; d2[k] = 0.f; }
  }
  // workgroup reduction of the 27 weight-gradient taps (+2 fp64 IN sums), fixed order
  __syncthreads();
  float* red = lds;                                        // [4 waves][27]
  double* redd = reinterpret_cast<double*>(lds + 112);     // [4 waves][2]
  const int wv = tid >> 6, ln = tid & 63;
#pragma unroll
  for (int t = 0; t < 27; ++t) {
    const float r = wave_sum(gw[t]);
    if (ln == 0) red[wv * 27 + t] = r;
  }
  if (MODE == 1) {
    const double r1 = wave_sum_d(s1), r2 = wave_sum_d(s2);
    if (ln == 0) { redd[wv * 2] = r1; redd[wv * 2 + 1] = r2; }
  }
  __syncthreads();
  if (tid < 27) {
    const float r = (red[tid] + red[27 + tid]) + (red[54 + tid] + red[81 + tid]);
    dw_part[((long long)c * N * nchunk + (long long)n * nchunk + chunk) * 27 + tid] = r;
  }
  if (MODE == 1 && tid >= 32 && tid < 34) {
    const int j = tid - 32;
    const double r = (redd[j] + redd[2 + j]) + (redd[4 + j] + redd[6 + j]);
    // in_part layout [c][n][chunk][2]
    in_part[(((long long)c * N + n) * nchunk + chunk) * 2 + j] = r;
  }
}

int pick_tz(int D) { return D <= 8 ? D : 4; }

}  // namespace

#define DW_DISPATCH_P(KERNEL, MODE, ...)                                               \
  do {                                                                                 \
    if (P <= 1) hipLaunchKernelGGL((KERNEL<MODE, 1>), __VA_ARGS__);                    \
    else if (P <= 2) hipLaunchKernelGGL((KERNEL<MODE, 2>), __VA_ARGS__);               \
    else if (P <= 3) hipLaunchKernelGGL((KERNEL<MODE, 3>), __VA_ARGS__);               \
    else if (P <= 4) hipLaunchKernelGGL((KERNEL<MODE, 4>), __VA_ARGS__);               \
    else if (P <= 6) hipLaunchKernelGGL((KERNEL<MODE, 6>), __VA_ARGS__);               \
    else if (P <= 9) hipLaunchKernelGGL((KERNEL<MODE, 9>), __VA_ARGS__);               \
    else if (P <= 12) hipLaunchKernelGGL((KERNEL<MODE, 12>), __VA_ARGS__);             \
    else hipLaunchKernelGGL((KERNEL<MODE, 16>), __VA_ARGS__);                          \
  } while (0)

extern "C" {

int l3u_dw3_nchunk(int D) { return (D + pick_tz(D) - 1) / pick_tz(D); }

int l3u_dw3_fwd(const float* x, long long x_nstride, const float* w, const float* rec, float* y,
                long long y_nstride, int N, int C, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && D > 0 && H > 0 && W > 0 && H * W <= 4096);
  const int TZ = pick_tz(D), nchunk = (D + TZ - 1) / TZ;
  const int P = (H * W + 255) / 256;
  const size_t lds = 2 * (size_t)(H + 2) * (W + 2) * sizeof(float);
  dim3 grid(N * C * nchunk), block(256);
  if (rec) DW_DISPATCH_P(dw3_fwd_kernel, 1, grid, block, lds, stream, x, x_nstride, w, rec, y, y_nstride, C, D, H, W, TZ, nchunk);
  else DW_DISPATCH_P(dw3_fwd_kernel, 0, grid, block, lds, stream, x, x_nstride, w, rec, y, y_nstride, C, D, H, W, TZ, nchunk);
  L3U_CHECK_LAUNCH();
}

int l3u_dw3_bwd(const float* dz, long long dz_nstride, const float* x, long long x_nstride,
                const float* w, const float* rec, float* dx, long long dx_nstride, int accumulate,
                float* dw_part, double* in_part, int N, int C, int D, int H, int W,
                hipStream_t stream) {
  L3U_REQUIRE(N > 0 && C > 0 && D > 0 && H > 0 && W > 0 && H * W <= 4096);
  L3U_REQUIRE(rec == nullptr || in_part != nullptr);
  const int TZ = pick_tz(D), nchunk = (D + TZ - 1) / TZ;
  const int P = (H * W + 255) / 256;
  size_t lds = 4 * (size_t)(H + 2) * (W + 2) * sizeof(float);
  if (lds < 128 * sizeof(float)) lds = 128 * sizeof(float);   // reduction scratch
  dim3 grid(N * C * nchunk), block(256);
  if (rec) DW_DISPATCH_P(dw3_bwd_kernel, 1, grid, block, lds, stream, dz, dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, accumulate, dw_part, in_part, N, C, D, H, W, TZ, nchunk);
  else DW_DISPATCH_P(dw3_bwd_kernel, 0, grid, block, lds, stream, dz, dz_nstride, x, x_nstride, w, rec, dx, dx_nstride, accumulate, dw_part, in_part, N, C, D, H, W, TZ, nchunk);
  L3U_CHECK_LAUNCH();
}

}  // extern "C"
