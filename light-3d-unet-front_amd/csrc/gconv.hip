// Grouped / dense 3x3x3 convolution (stride 1, zero padding 1, no bias): the
// use_depthwise_separable=False variants of ResidualBlock.conv1 / conv2:
//   GroupedConv3d(Cin, Cout, groups=G)  light_unet/models/unet3d.py:26-34 (chosen at :46-47, :57-58)
//   nn.Conv3d(Cin, Cout, 3, padding=1)  unet3d.py:49, :60 (G = 1; the first block always, :163-167)
// Per group the channel contraction is tiny (Cin/G x Cout/G = 2x2 .. 16x16 with the shipped
// channel plan and groups = 8), so this is not a dense GEMM and stays off MFMA: one thread per
// output voxel keeps CT output channels of one group in registers and walks the group's input
// channels x 27 taps (the taps' weights are wave-uniform: scalar loads; the input rows are
// coalesced along W and the 27-fold reuse is served by L1/L2).
//
//   gconv3_kernel   forward (and, with FLIP, the data gradient = the transposed conv)
//                   XF   input transformed on load: a = lrelu(scale*(y - mean) + shift) from the
//                        InstanceNorm record (IN1 + LeakyReLU + Dropout3d before conv2, :84-88),
//                        zero padding in the transformed domain
//                   EPI  0 store, 2 accumulate, 1 the IN-fused backward: dpre = o*k*lrelu'(pre)
//                        with pre from the saved pre-IN activation, plus the IN-backward partials
//                   STATS  (count, mean, M2) partials of the output per (n, channel, workgroup):
//                        the l3u_norm_src / l3u_in_finalize input format of l3u_pw_fwd
//   gconv3_wgrad_kernel  weight-gradient partials part[P][Cout][Cin/G][27], P = N * chunks
#include "common.h"
using namespace l3u;

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kGB = 256;      // output voxels per workgroup (one per thread)
constexpr int kWVPT = 8;      // voxels per thread of the weight-gradient kernel
constexpr int kKC = 16;       // input channels per LDS weight stage of the stencil kernel
constexpr int kWCO = 4;       // output channels per workgroup of the weight-gradient kernel

// Y[n][g*JG + j][v] = sum_{k < KG} sum_t Wt(g, j, k, t) * A[n][g*KG + k][v + off(t)]
//   FLIP = false (forward):        Wt = w[((g*JG + j)*KG + k)*27 + t]       (w: [Cout][Cin/G][27])
//   FLIP = true  (data gradient):  Wt = w[((g*KG + k)*JG + j)*27 + 26 - t]  (A = dY, Y = dX)
template <int CT, bool FLIP, bool XF, int EPI, bool STATS>
__global__ __launch_bounds__(256) void gconv3_kernel(
    const float* __restrict__ a, long long ans, const float* __restrict__ w,
    const float* __restrict__ rec_in, const float* __restrict__ rec_out,
    const float* __restrict__ ep, long long epns, float* __restrict__ y, long long yns,
    float* __restrict__ stat_part, double* __restrict__ in_part, int N, int G, int KG, int JG,
    int D, int H, int W) {
  __shared__ double redd[4];
  __shared__ float redf[4];
  const int S = D * H * W;
  const int nb = gridDim.x, bx = blockIdx.x;
  const int ntj = (JG + CT - 1) / CT;
  const int g = blockIdx.y / ntj, j0 = (blockIdx.y % ntj) * CT;
  const int n = blockIdx.z;
  const int v = bx * kGB + threadIdx.x;
  const bool act = v < S;
  const int vv = act ? v : 0;
  const int xx = vv % W, t1 = vv / W, yy = t1 % H, zz = t1 / H;
  const bool okz[3] = {zz > 0, true, zz < D - 1};
  const bool oky[3] = {yy > 0, true, yy < H - 1};
  const bool okx[3] = {xx > 0, true, xx < W - 1};
  float acc[CT];
#pragma unroll
  for (int j = 0; j < CT; ++j) acc[j] = 0.f;
  const float* an = a + (long long)n * ans;
  // the workgroup's weights, KC input channels at a time, staged in LDS as [k][t][j] (zero for
  // j >= JG): the CT weights of one (k, t) are one wave-uniform (broadcast) LDS vector read
  __shared__ __attribute__((aligned(16))) float wl[kKC * 27 * CT];
  for (int k0 = 0; k0 < KG; k0 += kKC) {
    const int kn = min(kKC, KG - k0);
    __syncthreads();
    for (int i = threadIdx.x; i < kn * 27 * CT; i += kGB) {
      const int kk = i / (27 * CT), rem = i - kk * 27 * CT, t = rem / CT, j = rem - t * CT;
      const int jj = j0 + j, k = k0 + kk;
      wl[i] = jj >= JG ? 0.f
                       : (FLIP ? w[((long long)(g * KG + k) * JG + jj) * 27 + 26 - t]
                               : w[((long long)(g * JG + jj) * KG + k) * 27 + t]);
    }
    __syncthreads();
    for (int kk = 0; kk < kn; ++kk) {
      const int ca = g * KG + k0 + kk;
      const float* ap = an + (long long)ca * S + vv;
      float mu = 0.f, sc = 1.f, sh = 0.f;
      if (XF) {
        const float* r = rec_in + ((long long)n * G * KG + ca) * kRec;
        mu = r[0]; sc = r[2]; sh = r[3];
      }
      const float* wk = wl + kk * 27 * CT;
      // the 27 neighbourhood loads first (latency), then tap by tap the CT weights from LDS;
      // the scheduling barrier keeps the weight reads of later taps from being hoisted (they
      // would hold 27 x CT registers)
      float val[27];
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const int dz = t / 9, dy = (t / 3) % 3, dx = t % 3;
        val[t] = 0.f;
        if (act && okz[dz] && oky[dy] && okx[dx]) val[t] = ap[((dz - 1) * H + (dy - 1)) * W + (dx - 1)];
      }
      if (XF) {
#pragma unroll
        for (int t = 0; t < 27; ++t) {
          const int dz = t / 9, dy = (t / 3) % 3, dx = t % 3;
          val[t] = (act && okz[dz] && oky[dy] && okx[dx]) ? lrelu(fmaf(sc, val[t] - mu, sh)) : 0.f;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const float v = val[t];
        if (CT % 4 == 0) {
#pragma unroll
          for (int j = 0; j < CT; j += 4) {
            const f4 w4 = *reinterpret_cast<const f4*>(wk + t * CT + j);
            acc[j] = fmaf(w4[0], v, acc[j]);
            acc[j + 1] = fmaf(w4[1], v, acc[j + 1]);
            acc[j + 2] = fmaf(w4[2], v, acc[j + 2]);
            acc[j + 3] = fmaf(w4[3], v, acc[j + 3]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < CT; ++j) acc[j] = fmaf(wk[t * CT + j], v, acc[j]);
        }
        asm volatile("" ::: "memory");   // no LDS weight read moves across taps
      }
    }
  }
  const int Cy = G * JG;
  const int cnt = min(kGB, S - bx * kGB);
#pragma unroll
  for (int j = 0; j < CT; ++j) {
    const int jj = j0 + j;
    if (jj >= JG) break;
    const int co = g * JG + jj;
    float* yp = y + (long long)n * yns + (long long)co * S;
    float o = acc[j];
    if (EPI == 1) {
      const float* r = rec_out + ((long long)n * Cy + co) * kRec;
      const float mu = r[0], rstd = r[1], sc = r[2], sh = r[3], kk = r[4];
      const float e = act ? ep[(long long)n * epns + (long long)co * S + v] : 0.f;
      const float dp = o * kk * lrelu_d(fmaf(sc, e - mu, sh));
      o = dp;
      const double s1 = block_sum256d(act ? (double)dp : 0.0, redd);
      const double s2 = block_sum256d(act ? (double)(dp * ((e - mu) * rstd)) : 0.0, redd);
      if (threadIdx.x == 0) {
        double* ip = in_part + (((long long)co * N + n) * nb + bx) * 2;
        ip[0] = s1;
        ip[1] = s2;
      }
    } else if (EPI == 2) {
      if (act) o += yp[v];
    }
    if (act) yp[v] = o;
    if (STATS) {
      const float mean = block_sum256(act ? o : 0.f, redf) / (float)cnt;
      const float d = act ? o - mean : 0.f;
      const float m2 = block_sum256(d * d, redf);
      if (threadIdx.x == 0) {
        float* sp = stat_part + (((long long)n * Cy + co) * nb + bx) * 3;
        sp[0] = (float)cnt;
        sp[1] = mean;
        sp[2] = m2;
      }
    }
  }
}

// part[(n*nbk + bx)][co][k][t] = sum over the chunk's voxels v of dY[n][co][v] * A[n][ci][v+off(t)],
// ci = (co / JG) * KG + k; A = x (XF 0) or lrelu(scale*(x-mean)+shift) (XF 1).  One workgroup per
// (chunk of kGB*kWVPT voxels, (group, k), n).  The chunk of A and its linear halo (one plane + one
// row + one voxel each side) is staged in LDS ONCE, transformed on the way in; the workgroup then
// walks the group's output channels CO at a time (each A neighbourhood read from LDS feeds CO
// channels) with a fixed-order workgroup reduction of CO x 27 taps per tile (deterministic).
template <bool XF, int CO>
__global__ __launch_bounds__(256) void gconv3_wgrad_kernel(
    const float* __restrict__ dy, long long dyns, const float* __restrict__ a, long long ans,
    const float* __restrict__ rec, float* __restrict__ part, int G, int KG, int JG, int D, int H,
    int W) {
  extern __shared__ float al[];            // [chunk + 2*halo] staged A, then [4][CO*27] reduction
  const int S = D * H * W, HW = H * W;
  const int halo = HW + W + 1, CH = kGB * kWVPT;
  const int nbk = gridDim.x, bx = blockIdx.x;
  const int g = blockIdx.y / KG, k = blockIdx.y % KG, ci = g * KG + k;
  const int n = blockIdx.z;
  const int v0 = bx * CH, lo = v0 - halo, len = min(CH, S - v0) + 2 * halo;
  const float* ap0 = a + (long long)n * ans + (long long)ci * S;
  float mu = 0.f, sc = 1.f, sh = 0.f;
  if (XF) {
    const float* r = rec + ((long long)n * G * KG + ci) * kRec;
    mu = r[0]; sc = r[2]; sh = r[3];
  }
  for (int i = threadIdx.x; i < len; i += kGB) {
    const int v = lo + i;
    float val = 0.f;
    if (v >= 0 && v < S) {
      val = ap0[v];
      if (XF) val = lrelu(fmaf(sc, val - mu, sh));
    }
    al[i] = val;
  }
  float* red = al + CH + 2 * halo;         // [4][CO*27]
  __syncthreads();
  const long long npair = (long long)G * JG * KG;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  for (int c0 = 0; c0 < JG; c0 += CO) {
    const float* dyp[CO];
#pragma unroll
    for (int j = 0; j < CO; ++j)
      dyp[j] = dy + (long long)n * dyns + (long long)(g * JG + min(c0 + j, JG - 1)) * S;
    float acc[CO][27];
#pragma unroll
    for (int j = 0; j < CO; ++j)
#pragma unroll
      for (int t = 0; t < 27; ++t) acc[j][t] = 0.f;
    for (int i = 0; i < kWVPT; ++i) {
      const int v = v0 + i * kGB + threadIdx.x;
      if (v >= S) break;
      float gv[CO];
#pragma unroll
      for (int j = 0; j < CO; ++j) gv[j] = dyp[j][v];
      const int xx = v % W, t1 = v / W, yy = t1 % H, zz = t1 / H;
      const bool okz[3] = {zz > 0, true, zz < D - 1};
      const bool oky[3] = {yy > 0, true, yy < H - 1};
      const bool okx[3] = {xx > 0, true, xx < W - 1};
      const float* ap = al + (v - lo);
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const int dz = t / 9, dyy = (t / 3) % 3, dx = t % 3;
        const float val = (okz[dz] && oky[dyy] && okx[dx]) ? ap[(dz - 1) * HW + (dyy - 1) * W + (dx - 1)] : 0.f;
#pragma unroll
        for (int j = 0; j < CO; ++j) acc[j][t] = fmaf(gv[j], val, acc[j][t]);
      }
    }
#pragma unroll
    for (int j = 0; j < CO; ++j)
#pragma unroll
      for (int t = 0; t < 27; ++t) {
        const float r = wave_sum(acc[j][t]);
        if (ln == 0) red[wv * CO * 27 + j * 27 + t] = r;
      }
    __syncthreads();
    for (int e = threadIdx.x; e < CO * 27; e += kGB) {
      const int j = e / 27, t = e - j * 27;
      if (c0 + j >= JG) continue;
      const float r = ((red[e] + red[CO * 27 + e]) + red[2 * CO * 27 + e]) + red[3 * CO * 27 + e];
      const long long pair = (long long)(g * JG + c0 + j) * KG + k;
      part[(((long long)n * nbk + bx) * npair + pair) * 27 + t] = r;
    }
    __syncthreads();
  }
}

int pick_ct(int JG) { return JG <= 1 ? 1 : (JG <= 2 ? 2 : (JG <= 4 ? 4 : (JG <= 8 ? 8 : 16))); }

#define GC_CT(CT_, ...)                                                            \
  do {                                                                             \
    if (CT_ == 1) hipLaunchKernelGGL((gconv3_kernel<1, __VA_ARGS__>), GC_ARGS);     \
    else if (CT_ == 2) hipLaunchKernelGGL((gconv3_kernel<2, __VA_ARGS__>), GC_ARGS);\
    else if (CT_ == 4) hipLaunchKernelGGL((gconv3_kernel<4, __VA_ARGS__>), GC_ARGS);\
    else if (CT_ == 8) hipLaunchKernelGGL((gconv3_kernel<8, __VA_ARGS__>), GC_ARGS);\
    else hipLaunchKernelGGL((gconv3_kernel<16, __VA_ARGS__>), GC_ARGS);            \
  } while (0)

}  // namespace

extern "C" {

int l3u_gconv3_nblocks(int S) { return (S + kGB - 1) / kGB; }

int l3u_gconv3_wgrad_nparts(int N, int S) { return N * ((S + kGB * kWVPT - 1) / (kGB * kWVPT)); }

int l3u_gconv3_fwd(const float* x, long long x_nstride, const float* w, const float* rec,
                   float* y, long long y_nstride, float* stat_part, int N, int Cin, int Cout,
                   int G, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && G > 0 && D > 0 && H > 0 && W > 0);
  L3U_REQUIRE(Cin % G == 0 && Cout % G == 0);
  L3U_REQUIRE((long long)D * H * W < (1ll << 31));
  const int S = D * H * W, KG = Cin / G, JG = Cout / G, CT = pick_ct(JG);
  dim3 grid(l3u_gconv3_nblocks(S), G * ((JG + CT - 1) / CT), N), block(kGB);
#define GC_ARGS grid, block, 0, stream, x, x_nstride, w, rec, nullptr, nullptr, 0, y, y_nstride, \
      stat_part, nullptr, N, G, KG, JG, D, H, W
  if (rec) {
    if (stat_part) GC_CT(CT, false, true, 0, true); else GC_CT(CT, false, true, 0, false);
  } else {
    if (stat_part) GC_CT(CT, false, false, 0, true); else GC_CT(CT, false, false, 0, false);
  }
#undef GC_ARGS
  L3U_CHECK_LAUNCH();
}

int l3u_gconv3_bwd_data(const float* dy, long long dy_nstride, const float* w, const float* rec,
                        const float* ep, long long ep_nstride, float* dx, long long dx_nstride,
                        int accumulate, double* in_part, int N, int Cin, int Cout, int G, int D,
                        int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && G > 0 && D > 0 && H > 0 && W > 0);
  L3U_REQUIRE(Cin % G == 0 && Cout % G == 0);
  L3U_REQUIRE((long long)D * H * W < (1ll << 31));
  L3U_REQUIRE(rec == nullptr || (ep != nullptr && in_part != nullptr && accumulate == 0));
  // the transposed conv: A = dY (Cout channels, KG = Cout/G per group), Y = dX (JG = Cin/G)
  const int S = D * H * W, KG = Cout / G, JG = Cin / G, CT = pick_ct(JG);
  dim3 grid(l3u_gconv3_nblocks(S), G * ((JG + CT - 1) / CT), N), block(kGB);
#define GC_ARGS grid, block, 0, stream, dy, dy_nstride, w, nullptr, rec, ep, ep_nstride, dx, \
      dx_nstride, nullptr, in_part, N, G, KG, JG, D, H, W
  if (rec) GC_CT(CT, true, false, 1, false);
  else if (accumulate) GC_CT(CT, true, false, 2, false);
  else GC_CT(CT, true, false, 0, false);
#undef GC_ARGS
  L3U_CHECK_LAUNCH();
}

int l3u_gconv3_bwd_weight(const float* dy, long long dy_nstride, const float* x,
                          long long x_nstride, const float* rec, float* part, int N, int Cin,
                          int Cout, int G, int D, int H, int W, hipStream_t stream) {
  L3U_REQUIRE(N > 0 && Cin > 0 && Cout > 0 && G > 0 && D > 0 && H > 0 && W > 0);
  L3U_REQUIRE(Cin % G == 0 && Cout % G == 0);
  const int S = D * H * W, KG = Cin / G, JG = Cout / G;
  const int co = JG >= kWCO ? kWCO : (JG >= 2 ? 2 : 1);
  L3U_REQUIRE((long long)D * H * W < (1ll << 31) && (long long)G * KG <= 65535);
  const int halo = H * W + W + 1;
  const size_t lds = ((size_t)kGB * kWVPT + 2 * halo + 4 * kWCO * 27) * sizeof(float);
  L3U_REQUIRE(lds <= 160 * 1024);
  dim3 grid(l3u_gconv3_wgrad_nparts(1, S), G * KG, N), block(kGB);
#define GW(X_, C_) hipLaunchKernelGGL((gconv3_wgrad_kernel<X_, C_>), grid, block, lds, stream, dy, \
      dy_nstride, x, x_nstride, rec, part, G, KG, JG, D, H, W)
  if (rec) { if (co == kWCO) GW(true, kWCO); else if (co == 2) GW(true, 2); else GW(true, 1); }
  else { if (co == kWCO) GW(false, kWCO); else if (co == 2) GW(false, 2); else GW(false, 1); }
#undef GW
  L3U_CHECK_LAUNCH();
}

}  // extern "C"
