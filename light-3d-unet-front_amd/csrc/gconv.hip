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
constexpr int kWVPT = 32;     // voxels per thread of the weight-gradient kernel (amortises its reductions)
constexpr int kKC = 16;       // input channels per LDS weight stage of the stencil kernel
constexpr int kWCO = 4;       // output channels per workgroup of the weight-gradient kernel

// Y[n][g*JG + j][v] = sum_{k < KG} sum_t Wt(g, j, k, t) * A[n][g*KG + k][v + off(t)]
//   FLIP = false (forward):        Wt = w[((g*JG + j)*KG + k)*27 + t]       (w: [Cout][Cin/G][27])
//   FLIP = true  (data gradient):  Wt = w[((g*KG + k)*JG + j)*27 + 26 - t]  (A = dY, Y = dX)
// LDSIN (one-block volumes, S <= 256: the 6^3 level): the group's KG input channels are staged in
// LDS first (transformed), one memory round trip instead of one per channel
template <int CT, bool FLIP, bool XF, int EPI, bool STATS, bool LDSIN = false>
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
  extern __shared__ float gin[];   // LDSIN: [KG][S]
  if (LDSIN) {
    for (int i = threadIdx.x; i < KG * S; i += kGB) {
      const int kk = i / S, vi = i - kk * S, ca = g * KG + kk;
      float u = an[(long long)ca * S + vi];
      if (XF) {
        const float* r = rec_in + ((long long)n * G * KG + ca) * kRec;
        u = lrelu(fmaf(r[2], u - r[0], r[3]));
      }
      gin[i] = u;
    }
  }
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
      const float* ap = LDSIN ? gin + (size_t)(k0 + kk) * S + vv : an + (long long)ca * S + vv;
      float mu = 0.f, sc = 1.f, sh = 0.f;
      if (XF && !LDSIN) {
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
      if (XF && !LDSIN) {
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

// ------------------------------------------------------------------------------------------------
// x-quad forms (W % 4 == 0: every shipped level).  A lane owns 4 consecutive voxels of one row and
// CT output channels (4 * CT accumulators); a wave owns one 256-voxel block (the unit of
// l3u_gconv3_nblocks, so the statistics / IN-backward partials keep their per-block layout).  Per
// input channel a lane reads its 3 x 3 neighbourhood rows as one float4 plus the two edge values
// (27 loads per 4 voxels instead of 4 x 27) and issues 27 x 4 x CT FMAs from them, in the voxel
// form's order (channel, then tap: the same sums); the CT weights of a tap are broadcast LDS reads.
//   LDSIN = false: the rows come straight from global memory (L1 / L2); a workgroup's waves are
//                  4 consecutive blocks.  Grid (ceil(nb / 4), G * slices, N).
//   LDSIN = true:  small volumes: the group's KG input channels are staged in LDS first (one
//                  memory round trip instead of one per channel), transformed on the way in; the
//                  workgroup's waves walk the blocks.  Grid (G * slices, N).
// Out-of-volume rows and edge values are loaded from clamped (valid) addresses and zeroed after
// the load (branch-free loads, the conv's zero padding in the transformed domain).
// ------------------------------------------------------------------------------------------------
template <int CT, bool FLIP, bool XF, int EPI, bool STATS, bool LDSIN>
__global__ __launch_bounds__(256) void gconv3q_kernel(
    const float* __restrict__ a, long long ans, const float* __restrict__ w,
    const float* __restrict__ rec_in, const float* __restrict__ rec_out,
    const float* __restrict__ ep, long long epns, float* __restrict__ y, long long yns,
    float* __restrict__ stat_part, double* __restrict__ in_part, int N, int G, int KG, int JG,
    int D, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) float gq_lds[];   // [kKC][27][CT] (+ [KG][S])
  const int S = D * H * W, nb = (S + kGB - 1) / kGB;
  const int ntj = (JG + CT - 1) / CT;
  const int gy = LDSIN ? blockIdx.x : blockIdx.y;
  const int g = gy / ntj, j0 = (gy % ntj) * CT;
  const int n = LDSIN ? blockIdx.y : blockIdx.z;
  const int nw = blockDim.x >> 6, wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  float* wl = gq_lds;
  float* ain = gq_lds + kKC * 27 * CT;
  const float* an = a + (long long)n * ans;
  const int Cy = G * JG;

  if (LDSIN) {   // the group's input channels, transformed (XF), S % 4 == 0
    const int S4 = S >> 2;
    for (int i = threadIdx.x; i < KG * S4; i += blockDim.x) {
      const int kk = i / S4, q = i - kk * S4, ca = g * KG + kk;
      f4 v = ldv4(an + (long long)ca * S + 4 * q);
      if (XF) {
        const float* r = rec_in + ((long long)n * G * KG + ca) * kRec;
        const float mu = r[0], sc = r[2], sh = r[3];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = lrelu(fmaf(sc, v[e] - mu, sh));
      }
      *reinterpret_cast<f4*>(ain + (size_t)kk * S + 4 * q) = v;
    }
  }
  auto stage_w = [&](int k0, int kn) {
    for (int i = threadIdx.x; i < kn * 27 * CT; i += blockDim.x) {
      const int kk = i / (27 * CT), rem = i - kk * 27 * CT, t = rem / CT, j = rem - t * CT;
      const int jj = j0 + j, k = k0 + kk;
      wl[i] = jj >= JG ? 0.f
                       : (FLIP ? w[((long long)(g * KG + k) * JG + jj) * 27 + 26 - t]
                               : w[((long long)(g * JG + jj) * KG + k) * 27 + t]);
    }
  };
  const bool one_stage = KG <= kKC;
  if (one_stage) stage_w(0, KG);
  __syncthreads();

  const int iters = LDSIN ? (nb + nw - 1) / nw : 1;
  for (int it = 0; it < iters; ++it) {
    const int b = LDSIN ? wave + nw * it : (int)blockIdx.x * nw + wave;
    const int v = b * kGB + 4 * l;
    const bool act = b < nb && v < S;
    const int vv = act ? v : 0;
    const int xx = vv % W, t1 = vv / W, yy = t1 % H, zz = t1 / H;
    int off[9];
    bool okr[9];
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const int z = zz + r / 3 - 1, yq = yy + r % 3 - 1;
      okr[r] = act && z >= 0 && z < D && yq >= 0 && yq < H;
      off[r] = (min(max(z, 0), D - 1) * H + min(max(yq, 0), H - 1)) * W + xx;
    }
    const bool okl = xx > 0, okrt = xx + 4 < W;
    const int dl = okl ? 1 : 0, dr = okrt ? 4 : 3;
    float acc[CT][4];
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[j][q] = 0.f;

    // the rows of input channel k: from LDS (LDSIN), or from global memory one channel ahead of
    // the FMAs (the next channel's loads are requested before this channel's FMAs)
    struct Rows { f4 m[9]; float lo[9], hi[9]; };
    auto fetch = [&](int k, Rows& R) {
      const float* base = LDSIN ? ain + (size_t)k * S : an + (long long)(g * KG + k) * S;
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        R.m[r] = ldv4(base + off[r]);
        R.lo[r] = base[off[r] - dl];
        R.hi[r] = base[off[r] + dr];
      }
    };
    Rows cur;
    if (!LDSIN) fetch(0, cur);
    for (int k = 0; k < KG; ++k) {
      const int kk = k % kKC;
      if (!one_stage && kk == 0) {
        __syncthreads();
        stage_w(k, min(kKC, KG - k));
        __syncthreads();
      }
      Rows nxt;
      if (LDSIN) fetch(k, cur);
      else fetch(min(k + 1, KG - 1), nxt);   // clamped: unconditional, no branch around the loads
      float mu = 0.f, sc = 1.f, sh = 0.f;
      if (XF && !LDSIN) {
        const float* r = rec_in + ((long long)n * G * KG + g * KG + k) * kRec;
        mu = r[0]; sc = r[2]; sh = r[3];
      }
      float v6[9][6];
#pragma unroll
      for (int r = 0; r < 9; ++r) {
        v6[r][0] = cur.lo[r];
        v6[r][1] = cur.m[r][0]; v6[r][2] = cur.m[r][1]; v6[r][3] = cur.m[r][2]; v6[r][4] = cur.m[r][3];
        v6[r][5] = cur.hi[r];
      }
#pragma unroll
      for (int r = 0; r < 9; ++r)
#pragma unroll
        for (int e = 0; e < 6; ++e) {
          const bool ok = okr[r] && (e > 0 || okl) && (e < 5 || okrt);
          float u = v6[r][e];
          if (XF && !LDSIN) u = lrelu(fmaf(sc, u - mu, sh));
          v6[r][e] = ok ? u : 0.f;
        }
      const float* wk = wl + kk * 27 * CT;
#pragma unroll
      for (int r = 0; r < 9; ++r)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int t = r * 3 + dx;
          if constexpr (CT % 4 == 0) {
#pragma unroll
            for (int j = 0; j < CT; j += 4) {
              const f4 w4 = *reinterpret_cast<const f4*>(wk + t * CT + j);
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                acc[j][q] = fmaf(w4[0], v6[r][q + dx], acc[j][q]);
                acc[j + 1][q] = fmaf(w4[1], v6[r][q + dx], acc[j + 1][q]);
                acc[j + 2][q] = fmaf(w4[2], v6[r][q + dx], acc[j + 2][q]);
                acc[j + 3][q] = fmaf(w4[3], v6[r][q + dx], acc[j + 3][q]);
              }
            }
          } else {
#pragma unroll
            for (int j = 0; j < CT; ++j) {
              const float wj = wk[t * CT + j];
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[j][q] = fmaf(wj, v6[r][q + dx], acc[j][q]);
            }
          }
        }
      if (!LDSIN) cur = nxt;
    }
    // epilogue per output channel; partials only for real blocks (b < nb)
    const int cnt = b < nb ? min(kGB, S - b * kGB) : 0;
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      const int jj = j0 + j;
      if (jj >= JG) continue;   // (not break: keeps acc[][] in registers)
      const int co = g * JG + jj;
      float* yp = y + (long long)n * yns + (long long)co * S + vv;
      f4 o = f4{acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
      if (EPI == 1) {
        const float* r = rec_out + ((long long)n * Cy + co) * kRec;
        const float mu = r[0], rstd = r[1], sc = r[2], sh = r[3], kk = r[4];
        const f4 e = ldv4(ep + (long long)n * epns + (long long)co * S + vv);
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float dp = o[q] * kk * lrelu_d(fmaf(sc, e[q] - mu, sh));
          o[q] = dp;
          s1 += act ? (double)dp : 0.0;
          s2 += act ? (double)(dp * ((e[q] - mu) * rstd)) : 0.0;
        }
        s1 = wave_sum_d(s1);
        s2 = wave_sum_d(s2);
        if (l == 0 && b < nb) {
          double* ip = in_part + (((long long)co * N + n) * nb + b) * 2;
          ip[0] = s1;
          ip[1] = s2;
        }
      } else if (EPI == 2) {
        if (act) o += ldv4(yp);
      }
      if (act) stv4(yp, o);
      if (STATS) {
        const float mean = wave_sum(act ? (o[0] + o[1]) + (o[2] + o[3]) : 0.f) / (float)max(cnt, 1);
        float m2 = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d = o[q] - mean;
          m2 = fmaf(d, d, m2);
        }
        m2 = wave_sum(act ? m2 : 0.f);
        if (l == 0 && b < nb) {
          float* sp = stat_part + (((long long)n * Cy + co) * nb + b) * 3;
          sp[0] = (float)cnt;
          sp[1] = mean;
          sp[2] = m2;
        }
      }
    }
  }
}

// Weight gradient, x-quad form (W % 4 == 0): part[(n*nbk + bx)][co][k][t] as gconv3_wgrad_kernel
// (same chunks of kGB * kWVPT voxels, same partial layout).  A workgroup owns (chunk, input
// channel, block of CO output channels, sample): it stages the chunk of A with a linear halo of
// one plane + one row + one voxel (rounded up to a quad, so every row read is an aligned
// ds_read_b128), IN-transformed once; a lane then owns voxel QUADS and, per quad, reads its 3 x 3
// neighbourhood rows from LDS and the CO dY quads from global memory, and issues 27 x 4 x CO FMAs;
// one fixed-order workgroup reduction of the 27 x CO sums ends the chunk.  The CO blocks are
// separate workgroups (grid.y), so the 1 -> 16 first conv gets 4x the workgroups of a co loop.
template <bool XF, int CO>
__global__ __launch_bounds__(256) void gconv3q_wgrad_kernel(
    const float* __restrict__ dy, long long dyns, const float* __restrict__ a, long long ans,
    const float* __restrict__ rec, float* __restrict__ part, int G, int KG, int JG, int D, int H,
    int W) {
  extern __shared__ __attribute__((aligned(16))) float wq_lds[];   // chunk + halo; [4][CO*27]
  const int S = D * H * W, HW = H * W, CH = kGB * kWVPT, QPT = kWVPT / 4;
  const int halo = (HW + W + 1 + 3) & ~3;
  const int nbk = gridDim.x, bx = blockIdx.x;
  const int ncb = (JG + CO - 1) / CO;
  const int cb = blockIdx.y % ncb, gk = blockIdx.y / ncb;
  const int g = gk / KG, k = gk % KG, ci = g * KG + k, c0 = cb * CO;
  const int n = blockIdx.z;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int v0 = bx * CH, lo = v0 - halo, len = min(CH, S - v0) + 2 * halo;
  float* al = wq_lds;
  float* red = wq_lds + CH + 2 * halo;
  {
    const float* ap = a + (long long)n * ans + (long long)ci * S;
    float mu = 0.f, sc = 1.f, sh = 0.f;
    if (XF) {
      const float* r = rec + ((long long)n * G * KG + ci) * kRec;
      mu = r[0]; sc = r[2]; sh = r[3];
    }
    // quads: lo, S and every in-volume quad boundary are multiples of 4 (W % 4 == 0)
    for (int i = 4 * threadIdx.x; i < len; i += 4 * kGB) {
      const int v = lo + i;
      f4 u = f4{0.f, 0.f, 0.f, 0.f};
      if (v >= 0 && v < S) {
        u = ldv4(ap + v);
        if (XF) {
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = lrelu(fmaf(sc, u[e] - mu, sh));
        }
      }
      *reinterpret_cast<f4*>(al + i) = u;
    }
  }
  const float* dyp[CO];
#pragma unroll
  for (int j = 0; j < CO; ++j)
    dyp[j] = dy + (long long)n * dyns + (long long)(g * JG + min(c0 + j, JG - 1)) * S;
  __syncthreads();
  float acc[CO][27];
#pragma unroll
  for (int j = 0; j < CO; ++j)
#pragma unroll
    for (int t = 0; t < 27; ++t) acc[j][t] = 0.f;
  for (int i = 0; i < QPT; ++i) {
    const int v = v0 + 4 * (i * kGB + threadIdx.x);
    const bool act = v < S;
    const int vv = act ? v : v0;
    const int xx = vv % W, t1 = vv / W, yy = t1 % H, zz = t1 / H;
    f4 gq[CO];
#pragma unroll
    for (int j = 0; j < CO; ++j) {
      gq[j] = ldv4(dyp[j] + vv);
      if (!act) gq[j] = f4{0.f, 0.f, 0.f, 0.f};
    }
    const bool okl = xx > 0, okrt = xx + 4 < W;
    const float* c = al + (vv - lo);
    float v6[9][6];
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const int dz = r / 3 - 1, dyy = r % 3 - 1;
      const bool okr = zz + dz >= 0 && zz + dz < D && yy + dyy >= 0 && yy + dyy < H;
      const float* rp = c + dz * HW + dyy * W;   // inside the staged range (halo >= HW + W + 1)
      const f4 m = *reinterpret_cast<const f4*>(rp);
      const float u[6] = {rp[-1], m[0], m[1], m[2], m[3], rp[4]};
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        const bool ok = okr && (e > 0 || okl) && (e < 5 || okrt);
        v6[r][e] = ok ? u[e] : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < 9; ++r)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int j = 0; j < CO; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[j][r * 3 + dx] = fmaf(gq[j][q], v6[r][q + dx], acc[j][r * 3 + dx]);
  }
#pragma unroll
  for (int j = 0; j < CO; ++j)
#pragma unroll
    for (int t = 0; t < 27; ++t) {
      const float r = wave_sum(acc[j][t]);
      if (ln == 0) red[wv * CO * 27 + j * 27 + t] = r;
    }
  __syncthreads();
  const long long npair = (long long)G * JG * KG;
  for (int e = threadIdx.x; e < CO * 27; e += kGB) {
    const int j = e / 27, t = e - j * 27;
    if (c0 + j >= JG) continue;
    const float r = ((red[e] + red[CO * 27 + e]) + red[2 * CO * 27 + e]) + red[3 * CO * 27 + e];
    const long long pair = (long long)(g * JG + c0 + j) * KG + k;
    part[(((long long)n * nbk + bx) * npair + pair) * 27 + t] = r;
  }
}

// Weight gradient of one-block volumes (S <= 256, the 6^3 level; one chunk, so the partial is the
// whole sum): the sample's A channel (transformed) and its group's JG dY channels are staged in
// LDS, and a thread owns whole outputs (co, t), summing the S voxels in order -- no cross-lane
// reduction (the reduction of the voxel form took most of its time at 6^3)
template <bool XF>
__global__ __launch_bounds__(256) void gconv3s_wgrad_kernel(
    const float* __restrict__ dy, long long dyns, const float* __restrict__ a, long long ans,
    const float* __restrict__ rec, float* __restrict__ part, int G, int KG, int JG, int D, int H,
    int W) {
  // LDS: A zero-padded to (D+2)(H+2)(W+2) (no bounds tests in the voxel loop), the padded index
  // of every voxel, then the group's JG dY channels
  extern __shared__ float sw_lds[];
  const int S = D * H * W, W2 = W + 2, P2 = (H + 2) * W2, SP = (D + 2) * P2;
  const int g = blockIdx.y / KG, k = blockIdx.y % KG, ci = g * KG + k;
  const int n = blockIdx.z;
  float* al = sw_lds;
  int* pidx = reinterpret_cast<int*>(sw_lds + SP);
  float* gl = sw_lds + SP + S;
  const float* ap = a + (long long)n * ans + (long long)ci * S;
  float mu = 0.f, sc = 1.f, sh = 0.f;
  if (XF) {
    const float* r = rec + ((long long)n * G * KG + ci) * kRec;
    mu = r[0]; sc = r[2]; sh = r[3];
  }
  for (int i = threadIdx.x; i < SP; i += blockDim.x) al[i] = 0.f;
  __syncthreads();
  for (int i = threadIdx.x; i < S; i += blockDim.x) {
    const int x = i % W, t1 = i / W, yq = t1 % H, z = t1 / H;
    const int pi = ((z + 1) * (H + 2) + yq + 1) * W2 + x + 1;
    float u = ap[i];
    if (XF) u = lrelu(fmaf(sc, u - mu, sh));
    al[pi] = u;
    pidx[i] = pi;
  }
  const float* dyn = dy + (long long)n * dyns + (long long)g * JG * S;
  for (int i = threadIdx.x; i < JG * S; i += blockDim.x) gl[i] = dyn[i];   // the group's channels
  __syncthreads();
  const long long npair = (long long)G * JG * KG;
  for (int e = threadIdx.x; e < JG * 27; e += blockDim.x) {
    const int j = e / 27, t = e - j * 27;
    const int off = (t / 9 - 1) * P2 + ((t / 3) % 3 - 1) * W2 + (t % 3 - 1);
    const float* gj = gl + j * S;
    // four interleaved partial sums (independent LDS loads in flight), combined in a fixed order
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int v = 0;
    for (; v + 4 <= S; v += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = fmaf(gj[v + u], al[pidx[v + u] + off], acc[u]);
    }
    for (; v < S; ++v) acc[0] = fmaf(gj[v], al[pidx[v] + off], acc[0]);
    const long long pair = (long long)(g * JG + j) * KG + k;
    part[((long long)n * npair + pair) * 27 + t] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
}

int pick_ct(int JG) { return JG <= 1 ? 1 : (JG <= 2 ? 2 : (JG <= 4 ? 4 : (JG <= 8 ? 8 : 16))); }

// x-quad dispatch: LDS-staged input for small volumes, global rows otherwise
constexpr int kQLdsMaxS = 4096;
#ifndef L3U_GQ_CTMAX
#define L3U_GQ_CTMAX 8
#endif
constexpr int kGqCtMax = L3U_GQ_CTMAX;   // output channels per lane of the global-row form
struct QPlan {
  bool ok, ldsin;
  int ct;
  size_t lds;
  dim3 grid, block;
};
QPlan q_plan(int N, int G, int KG, int JG, int D, int H, int W) {
  QPlan p{};
  const int S = D * H * W, nb = (S + kGB - 1) / kGB;
  p.ok = W % 4 == 0;
  if (!p.ok) return p;
  const int ctmax = min(pick_ct(JG), kGqCtMax);
  const size_t in_bytes = (size_t)KG * S * sizeof(float);
  p.ldsin = S <= kQLdsMaxS && in_bytes + (size_t)kKC * 27 * 8 * sizeof(float) <= 144 * 1024;
  if (p.ldsin) {
    // the largest CT that still gives >= 256 workgroups (one per (group, slice, sample))
    int ct = ctmax;
    while (ct > 1 && (long long)G * ((JG + ct - 1) / ct) * N < 256) ct >>= 1;
    p.ct = ct;
    p.grid = dim3(G * ((JG + ct - 1) / ct), N);
    p.block = dim3(64 * min(4, nb));
    p.lds = in_bytes + (size_t)kKC * 27 * ct * sizeof(float);
  } else {
    p.ct = ctmax;
    p.grid = dim3((nb + 3) / 4, G * ((JG + ctmax - 1) / ctmax), N);
    p.block = dim3(256);
    p.lds = (size_t)kKC * 27 * ctmax * sizeof(float);
  }
  return p;
}
#define GQ_CT(CT_, ...)                                                                   \
  do {                                                                                    \
    if (CT_ == 1) hipLaunchKernelGGL((gconv3q_kernel<1, __VA_ARGS__>), GQ_ARGS);           \
    else if (CT_ == 2) hipLaunchKernelGGL((gconv3q_kernel<2, __VA_ARGS__>), GQ_ARGS);      \
    else if (CT_ == 4) hipLaunchKernelGGL((gconv3q_kernel<4, __VA_ARGS__>), GQ_ARGS);      \
    else if (CT_ == 8 || kGqCtMax < 16) hipLaunchKernelGGL((gconv3q_kernel<8, __VA_ARGS__>), GQ_ARGS); \
    else hipLaunchKernelGGL((gconv3q_kernel<kGqCtMax, __VA_ARGS__>), GQ_ARGS);             \
  } while (0)

// one-block volumes with W % 4 != 0 (6^3): the voxel kernel with LDS-staged input, CT small
// enough for >= 256 workgroups
struct SPlan { bool ok; int ct; size_t lds; dim3 grid; };
SPlan s_plan(int N, int G, int KG, int JG, int D, int H, int W) {
  SPlan p{};
  const int S = D * H * W;
  p.ok = S <= kGB && (size_t)KG * S * sizeof(float) <= 64 * 1024;
  if (!p.ok) return p;
  int ct = pick_ct(JG);
  while (ct > 1 && (long long)G * ((JG + ct - 1) / ct) * N < 256) ct >>= 1;
  p.ct = ct;
  p.grid = dim3(1, G * ((JG + ct - 1) / ct), N);
  p.lds = (size_t)KG * S * sizeof(float);
  return p;
}

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
  const QPlan qp = q_plan(N, G, KG, JG, D, H, W);
  if (qp.ok) {
#define GQ_ARGS qp.grid, qp.block, qp.lds, stream, x, x_nstride, w, rec, nullptr, nullptr, 0, y, \
      y_nstride, stat_part, nullptr, N, G, KG, JG, D, H, W
#define GQ_L(L_) do { if (rec) { if (stat_part) GQ_CT(qp.ct, false, true, 0, true, L_); else GQ_CT(qp.ct, false, true, 0, false, L_); } \
                      else { if (stat_part) GQ_CT(qp.ct, false, false, 0, true, L_); else GQ_CT(qp.ct, false, false, 0, false, L_); } } while (0)
    if (qp.ldsin) GQ_L(true); else GQ_L(false);
#undef GQ_L
#undef GQ_ARGS
    L3U_CHECK_LAUNCH();
  }
  const SPlan sp = s_plan(N, G, KG, JG, D, H, W);
  if (sp.ok) {
#define GC_ARGS sp.grid, dim3(kGB), sp.lds, stream, x, x_nstride, w, rec, nullptr, nullptr, 0, y, \
      y_nstride, stat_part, nullptr, N, G, KG, JG, D, H, W
    if (rec) {
      if (stat_part) GC_CT(sp.ct, false, true, 0, true, true); else GC_CT(sp.ct, false, true, 0, false, true);
    } else {
      if (stat_part) GC_CT(sp.ct, false, false, 0, true, true); else GC_CT(sp.ct, false, false, 0, false, true);
    }
#undef GC_ARGS
    L3U_CHECK_LAUNCH();
  }
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
  const QPlan qp = q_plan(N, G, KG, JG, D, H, W);
  if (qp.ok) {
#define GQ_ARGS qp.grid, qp.block, qp.lds, stream, dy, dy_nstride, w, nullptr, rec, ep, ep_nstride, \
      dx, dx_nstride, nullptr, in_part, N, G, KG, JG, D, H, W
#define GQ_L(L_) do { if (rec) GQ_CT(qp.ct, true, false, 1, false, L_); \
                      else if (accumulate) GQ_CT(qp.ct, true, false, 2, false, L_); \
                      else GQ_CT(qp.ct, true, false, 0, false, L_); } while (0)
    if (qp.ldsin) GQ_L(true); else GQ_L(false);
#undef GQ_L
#undef GQ_ARGS
    L3U_CHECK_LAUNCH();
  }
  const SPlan sp = s_plan(N, G, KG, JG, D, H, W);
  if (sp.ok) {
#define GC_ARGS sp.grid, dim3(kGB), sp.lds, stream, dy, dy_nstride, w, nullptr, rec, ep, ep_nstride, \
      dx, dx_nstride, nullptr, in_part, N, G, KG, JG, D, H, W
    if (rec) GC_CT(sp.ct, true, false, 1, false, true);
    else if (accumulate) GC_CT(sp.ct, true, false, 2, false, true);
    else GC_CT(sp.ct, true, false, 0, false, true);
#undef GC_ARGS
    L3U_CHECK_LAUNCH();
  }
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
  const size_t slds = ((size_t)(D + 2) * (H + 2) * (W + 2) + (size_t)(JG + 1) * S) * sizeof(float);
  if (S <= kGB && slds <= 64 * 1024) {   // one chunk
    dim3 grid(1, G * KG, N), block(kGB);
    const size_t lds = slds;
    if (rec) hipLaunchKernelGGL((gconv3s_wgrad_kernel<true>), grid, block, lds, stream, dy, dy_nstride, x,
                                x_nstride, rec, part, G, KG, JG, D, H, W);
    else hipLaunchKernelGGL((gconv3s_wgrad_kernel<false>), grid, block, lds, stream, dy, dy_nstride, x,
                            x_nstride, rec, part, G, KG, JG, D, H, W);
    L3U_CHECK_LAUNCH();
  }
  if (W % 4 == 0) {
    const int halo4 = (H * W + W + 1 + 3) & ~3;
    const size_t qlds = ((size_t)kGB * kWVPT + 2 * halo4 + 4 * kWCO * 27) * sizeof(float);
    L3U_REQUIRE(qlds <= 160 * 1024 && (long long)G * KG * ((JG + co - 1) / co) <= 65535);
    dim3 grid(l3u_gconv3_wgrad_nparts(1, S), G * KG * ((JG + co - 1) / co), N), block(kGB);
#define GQW(X_, C_) hipLaunchKernelGGL((gconv3q_wgrad_kernel<X_, C_>), grid, block, qlds, stream, dy, \
      dy_nstride, x, x_nstride, rec, part, G, KG, JG, D, H, W)
    if (rec) { if (co == kWCO) GQW(true, kWCO); else if (co == 2) GQW(true, 2); else GQW(true, 1); }
    else { if (co == kWCO) GQW(false, kWCO); else if (co == 2) GQW(false, 2); else GQW(false, 1); }
#undef GQW
    L3U_CHECK_LAUNCH();
  }
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
