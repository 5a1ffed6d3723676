// Whole-volume sliding-window inference, the device halves of sliding_window_inference_3d
// (light_unet/utils.py:11-139):
//   window_gather  batch of B windows [B][1][pd][ph][pw] cut out of the volume, zero padding
//                  past the volume edge (utils.py:96-113, np.pad constant 0)
//   window_blend   prob = sum_w pred_w * imp / sum_w imp over the windows covering each voxel,
//                  accumulated in the reference's window order (z, y, x loops, utils.py:88-132)
//                  with separate fp32 multiply and add (no FMA contraction), then prob/count
//                  where count > 0 (utils.py:135) -- the same float32 operation sequence as the
//                  reference's numpy accumulation, done by one thread per voxel (deterministic:
//                  no atomics, no order dependence on the batching)
#include "common.h"
using namespace l3u;

namespace {

__global__ __launch_bounds__(256) void window_gather_kernel(
    const float* __restrict__ img, int D, int H, int W, const int* __restrict__ pos, int pd,
    int ph, int pw, float* __restrict__ out) {
  const int b = blockIdx.y;
  const long long P = (long long)pd * ph * pw;
  const int z0 = pos[3 * b], y0 = pos[3 * b + 1], x0 = pos[3 * b + 2];
  float* o = out + (long long)b * P;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < P; i += (long long)gridDim.x * 256) {
    const int k = (int)(i % pw), t = (int)(i / pw), j = t % ph, l = t / ph;
    const int z = z0 + l, y = y0 + j, x = x0 + k;
    o[i] = (z < D && y < H && x < W) ? img[((long long)z * H + y) * W + x] : 0.f;
  }
}

// covering window range [lo, hi) along one axis: positions ascending, window at p covers
// [p, p + len)
L3U_DEV void cover(const int* __restrict__ p, int n, int len, int v, int& lo, int& hi) {
  lo = n;
  hi = 0;
  for (int i = 0; i < n; ++i) {
    if (p[i] <= v && v < p[i] + len) {
      lo = min(lo, i);
      hi = max(hi, i + 1);
    }
  }
}

__global__ __launch_bounds__(256) void window_blend_kernel(
    const float* __restrict__ preds, const int* __restrict__ zp, int nz, const int* __restrict__ yp,
    int ny, const int* __restrict__ xp, int nx, const float* __restrict__ imp, int D, int H, int W,
    int pd, int ph, int pw, float* __restrict__ prob) {
  const long long V = (long long)D * H * W, P = (long long)pd * ph * pw;
  for (long long v = blockIdx.x * 256ll + threadIdx.x; v < V; v += (long long)gridDim.x * 256) {
    const int x = (int)(v % W), t = (int)(v / W), y = t % H, z = t / H;
    int z_lo, z_hi, y_lo, y_hi, x_lo, x_hi;
    cover(zp, nz, pd, z, z_lo, z_hi);
    cover(yp, ny, ph, y, y_lo, y_hi);
    cover(xp, nx, pw, x, x_lo, x_hi);
    float acc = 0.f, cnt = 0.f;
    for (int iz = z_lo; iz < z_hi; ++iz)
      for (int iy = y_lo; iy < y_hi; ++iy)
        for (int ix = x_lo; ix < x_hi; ++ix) {
          const long long li = ((long long)(z - zp[iz]) * ph + (y - yp[iy])) * pw + (x - xp[ix]);
          const long long win = ((long long)iz * ny + iy) * nx + ix;
          const float wgt = imp[li];
          acc = __fadd_rn(acc, __fmul_rn(preds[win * P + li], wgt));
          cnt = __fadd_rn(cnt, wgt);
        }
    prob[v] = cnt > 0.f ? __fdiv_rn(acc, cnt) : acc;
  }
}

}  // namespace

extern "C" {

int l3u_window_gather(const float* img, int D, int H, int W, const int* pos, int B, int pd, int ph,
                      int pw, float* out, hipStream_t stream) {
  L3U_REQUIRE(D > 0 && H > 0 && W > 0 && B > 0 && pd > 0 && ph > 0 && pw > 0);
  const long long P = (long long)pd * ph * pw;
  long long nb = (P + 1023) / 1024;
  if (nb > 1024) nb = 1024;
  hipLaunchKernelGGL(window_gather_kernel, dim3((int)nb, B), dim3(256), 0, stream, img, D, H, W, pos,
                     pd, ph, pw, out);
  L3U_CHECK_LAUNCH();
}

int l3u_window_blend(const float* preds, const int* zpos, int nz, const int* ypos, int ny,
                     const int* xpos, int nx, const float* imp, int D, int H, int W, int pd, int ph,
                     int pw, float* prob, hipStream_t stream) {
  L3U_REQUIRE(D > 0 && H > 0 && W > 0 && nz > 0 && ny > 0 && nx > 0);
  const long long V = (long long)D * H * W;
  long long nb = (V + 255) / 256;
  if (nb > 65536) nb = 65536;
  hipLaunchKernelGGL(window_blend_kernel, dim3((int)nb), dim3(256), 0, stream, preds, zpos, nz, ypos,
                     ny, xpos, nx, imp, D, H, W, pd, ph, pw, prob);
  L3U_CHECK_LAUNCH();
}

}  // extern "C"
