// Training-patch extraction and augmentation on the device, a batch of patches per launch pair.
// Replaces the per-sample host numpy / scipy work of PatchDataset.__getitem__
// (light_unet/datasets/patch_dataset.py:114-220): crop (:136-154), flip, rotation
// (scipy.ndimage.rotate, reshape=False, order 1 image / 0 label, mode 'constant'), scale
// (scipy.ndimage.zoom + centre crop / end pad), intensity shift and gaussian noise, each clipped to
// [0, 1] as the reference does.  The random draws stay on the host (light_unet/patches.py makes the
// reference's own RNG calls, in its order); the kernels get one l3u_aug_param per patch.
//
// Two passes, because the reference interpolates twice (zoom of the rotated patch):
//   aug_rotate: R = rotate(flip(crop(volume)))   — bilinear / nearest in the rotation plane
//   aug_zoom:   out = noise(shift(fit(zoom(R))))  — trilinear / nearest, then the clips
// Coordinates and interpolation weights are float64, accumulated in scipy's C order, and every
// intermediate is rounded to float32 where the reference's arrays are float32 (rotate / zoom
// outputs); the noise sum stays float64 until the final store (the reference's noise is a float64
// array).  One thread per output voxel; the patch volume (48^3 x B) is small and L2-resident.
#include "common.h"
using namespace l3u;

namespace {

// F[v] = the flipped, zero-padded crop at patch index v (patch_dataset.py:136-166)
L3U_DEV float crop_at(const float* __restrict__ vol, const l3u_aug_param& p, int z, int y, int x) {
  if (p.flip == 0) z = p.pz - 1 - z;
  else if (p.flip == 1) y = p.py - 1 - y;
  else if (p.flip == 2) x = p.px - 1 - x;
  const int sz = p.z0 + z, sy = p.y0 + y, sx = p.x0 + x;
  if (sz >= p.sd || sy >= p.sh || sx >= p.sw) return 0.f;   // the end padding of the crop
  return vol[((long long)sz * p.sh + sy) * p.sw + sx];
}

__global__ __launch_bounds__(256) void aug_rotate_kernel(const l3u_aug_param* __restrict__ prm,
                                                         float* __restrict__ rimg,
                                                         float* __restrict__ rlab, int B, long long P) {
  const long long n = (long long)B * P;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int b = (int)(i / P);
    const l3u_aug_param& p = prm[b];
    const long long v = i - (long long)b * P;
    const float* image = p.image;
    const float* label = p.label;
    int c[3] = {(int)(v / ((long long)p.py * p.px)), (int)((v / p.px) % p.py), (int)(v % p.px)};
    float oi, ol;
    if (p.rot_a0 < 0) {
      oi = crop_at(image, p, c[0], c[1], c[2]);
      ol = crop_at(label, p, c[0], c[1], c[2]);
    } else {
      const int a0 = p.rot_a0, a1 = p.rot_a1;
      const int dims[3] = {p.pz, p.py, p.px};
      // in = R @ out + offset (scipy affine_transform: offset first, then the row products)
      const double o0 = c[a0], o1 = c[a1];
      const double q0 = p.rot_off0 + p.rot_c * o0 + p.rot_s * o1;
      const double q1 = p.rot_off1 + (-p.rot_s) * o0 + p.rot_c * o1;
      const bool inside = q0 >= 0.0 && q0 <= dims[a0] - 1 && q1 >= 0.0 && q1 <= dims[a1] - 1;
      oi = ol = 0.f;
      if (inside) {
        int k[3] = {c[0], c[1], c[2]};
        // order 0 (label): floor(q + 0.5)
        k[a0] = (int)floor(q0 + 0.5);
        k[a1] = (int)floor(q1 + 0.5);
        ol = crop_at(label, p, k[0], k[1], k[2]);
        // order 1 (image): bilinear, weights (1 - t, t), C-order accumulation in float64
        const double f0 = floor(q0), f1 = floor(q1), t0 = q0 - f0, t1 = q1 - f1;
        const int l0 = (int)f0, l1 = (int)f1;
        const int h0 = min(l0 + 1, dims[a0] - 1), h1 = min(l1 + 1, dims[a1] - 1);
        double acc = 0.0;
#pragma unroll
        for (int cr = 0; cr < 4; ++cr) {
          const int b0 = cr >> 1, b1 = cr & 1;
          const double w = (b0 ? t0 : 1.0 - t0) * (b1 ? t1 : 1.0 - t1);
          k[a0] = b0 ? h0 : l0;
          k[a1] = b1 ? h1 : l1;
          acc += w * (double)crop_at(image, p, k[0], k[1], k[2]);
        }
        oi = (float)acc;
      }
    }
    rimg[i] = oi;
    rlab[i] = ol;
  }
}

__global__ __launch_bounds__(256) void aug_zoom_kernel(const float* __restrict__ rimg,
                                                       const float* __restrict__ rlab,
                                                       const l3u_aug_param* __restrict__ prm,
                                                       const double* __restrict__ noise,
                                                       float* __restrict__ oimg,
                                                       float* __restrict__ olab, int B, long long P) {
  const long long n = (long long)B * P;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int b = (int)(i / P);
    const l3u_aug_param& p = prm[b];
    const long long v = i - (long long)b * P;
    const int dims[3] = {p.pz, p.py, p.px};
    const int o[3] = {(int)(v / ((long long)p.py * p.px)), (int)((v / p.px) % p.py), (int)(v % p.px)};
    const float* ri = rimg + (long long)b * P;
    const float* rl = rlab + (long long)b * P;
    float vi, vl;
    if (!p.zoom) {
      vi = ri[v];
      vl = rl[v];
    } else {
      // fit (patch_dataset.py:183-206): centre crop of a larger zoomed volume, end pad of a smaller
      bool pad = false;
      double q[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const int u = o[d] + p.zst[d];
        pad |= u >= p.zs[d];
        q[d] = (double)u * p.zf[d];   // scipy zoom_shift: out * (in - 1) / (out - 1)
      }
      vi = vl = 0.f;
      bool inside = !pad;
#pragma unroll
      for (int d = 0; d < 3; ++d) inside &= q[d] >= 0.0 && q[d] <= dims[d] - 1;
      if (inside) {
        int k[3], lo[3], hi[3];
        double t[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          k[d] = (int)floor(q[d] + 0.5);
          const double f = floor(q[d]);
          t[d] = q[d] - f;
          lo[d] = (int)f;
          hi[d] = min(lo[d] + 1, dims[d] - 1);
        }
        vl = rl[((long long)k[0] * dims[1] + k[1]) * dims[2] + k[2]];
        double acc = 0.0;
#pragma unroll
        for (int cr = 0; cr < 8; ++cr) {
          const int b0 = cr >> 2, b1 = (cr >> 1) & 1, b2 = cr & 1;
          const double w = ((b0 ? t[0] : 1.0 - t[0]) * (b1 ? t[1] : 1.0 - t[1])) * (b2 ? t[2] : 1.0 - t[2]);
          acc += w * (double)ri[((long long)(b0 ? hi[0] : lo[0]) * dims[1] + (b1 ? hi[1] : lo[1])) * dims[2] +
                                (b2 ? hi[2] : lo[2])];
        }
        vi = (float)acc;
      }
    }
    if (p.shift_on) vi = fminf(fmaxf(vi + p.shift, 0.f), 1.f);   // float32 image + scalar, clip
    if (p.noise_on && noise) {
      const double s = (double)vi + noise[i];                       // float64 noise array
      vi = (float)fmin(fmax(s, 0.0), 1.0);
    }
    oimg[i] = vi;
    olab[i] = vl;
  }
}

int blocks_for(long long n) {
  const long long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" int l3u_aug_patches(const l3u_aug_param* params, int B, int pz, int py, int px,
                               const double* noise, float* tmp_img, float* tmp_lab, float* out_img,
                               float* out_lab, hipStream_t stream) {
  L3U_REQUIRE(params && B > 0 && pz > 0 && py > 0 && px > 0 && tmp_img && tmp_lab && out_img && out_lab);
  const long long P = (long long)pz * py * px, n = (long long)B * P;
  hipLaunchKernelGGL(aug_rotate_kernel, dim3(blocks_for(n)), dim3(256), 0, stream, params, tmp_img,
                     tmp_lab, B, P);
  hipLaunchKernelGGL(aug_zoom_kernel, dim3(blocks_for(n)), dim3(256), 0, stream, tmp_img, tmp_lab,
                     params, noise, out_img, out_lab, B, P);
  L3U_CHECK_LAUNCH();
}
