// Mask-aligned batch augmentation on the device for gfx950: the reference's AugmentationTransform
// (train_cswinunet_segmentation.py cswin:20-87: horizontal flip, vertical flip, rotation by a
// multiple of 90 degrees, random crop resized back with bilinear interpolation) followed by the
// dataset's normalisation and layout change (cswin:166-173: /255, HWC -> CHW), for a whole batch in
// one pass: one thread per output pixel computes its source position through crop -> rotate ->
// flips backwards, samples the uint8 image (3 channels) and mask bilinearly, and writes fp32.
// Per-image parameters are drawn on the host (csu.data.AugmentationTransform.draw, the
// reference's np.random call order) and passed as a small device table.
#include "common.hpp"

namespace csu {
namespace {

constexpr int NT = 256;

// pixel (y, x) of the rotated/flipped square image -> pixel of the stored image
__device__ __forceinline__ void src_of(int S, int hflip, int vflip, int rot, int y, int x, int* sy, int* sx) {
    // inverse rotation (rot = clockwise quarter turns applied after the flips)
    int a = y, b = x;
    if (rot == 1) { a = S - 1 - x; b = y; }          // R[y][x] = F[S-1-x][y]   (90 clockwise)
    else if (rot == 2) { a = S - 1 - y; b = S - 1 - x; }
    else if (rot == 3) { a = x; b = S - 1 - y; }     // R[y][x] = F[x][S-1-y]   (90 counter-clockwise)
    // inverse flips: F = vflip(hflip(I))
    if (vflip) a = S - 1 - a;
    if (hflip) b = S - 1 - b;
    *sy = a;
    *sx = b;
}

// bilinear source coordinate of output index o for an n -> m resize (half-pixel centres, clamped
// at the borders): integer part and weight of the upper neighbour
__device__ __forceinline__ void lin(int o, int n, int m, int* i0, int* i1, float* f) {
    float s = ((float)o + 0.5f) * ((float)n / (float)m) - 0.5f;
    if (s < 0.f) s = 0.f;
    int i = (int)s;
    if (i > n - 1) i = n - 1;
    *f = s - (float)i;
    *i0 = i;
    *i1 = i + 1 < n ? i + 1 : n - 1;
}

__global__ __launch_bounds__(NT) void augment_kernel(int B, int S, const uint8_t* __restrict__ img,
                                                     const uint8_t* __restrict__ mask, const int* __restrict__ prm,
                                                     float* __restrict__ oimg, float* __restrict__ omask) {
    const long n = (long)B * S * S;
    for (long q = (long)blockIdx.x * NT + threadIdx.x; q < n; q += (long)gridDim.x * NT) {
        const int b = (int)(q / ((long)S * S));
        const int r = (int)(q - (long)b * S * S), oy = r / S, ox = r - oy * S;
        const int* p = prm + 7 * b;   // hflip, vflip, rot, top, left, crop_h, crop_w
        int y0, y1, x0, x1;
        float fy, fx;
        lin(oy, p[5], S, &y0, &y1, &fy);
        lin(ox, p[6], S, &x0, &x1, &fx);
        const int cy[2] = {p[3] + y0, p[3] + y1}, cx[2] = {p[4] + x0, p[4] + x1};
        const float wy[2] = {1.f - fy, fy}, wx[2] = {1.f - fx, fx};
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                int sy, sx;
                src_of(S, p[0], p[1], p[2], cy[i], cx[j], &sy, &sx);
                const long pix = ((long)b * S + sy) * S + sx;
                const float w = wy[i] * wx[j];
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[c] += w * (float)img[pix * 3 + c];
                acc[3] += w * (float)mask[pix];
            }
        // uint8 results as the reference's resize yields them (round half up, as cv2's fixed-point resize), then / 255 (an IEEE division, as the reference's float32 / 255.0; not a reciprocal multiply)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            oimg[(((long)b * 3 + c) * S + oy) * S + ox] = fminf(fmaxf(floorf(acc[c] + 0.5f), 0.f), 255.f) / 255.f;
        omask[((long)b * S + oy) * S + ox] = fminf(fmaxf(floorf(acc[3] + 0.5f), 0.f), 255.f) / 255.f;
    }
}

}  // namespace
}  // namespace csu

using namespace csu;

extern "C" int csu_augment_batch(int B, int S, const void* img, const void* mask, const int* params, float* out_img,
                                 float* out_mask, void* stream) {
    if (B < 1 || S < 1 || !img || !mask || !params || !out_img || !out_mask) return fail(CSU_E_ARG, "augment_batch: bad args");
    const long n = (long)B * S * S;
    const long g = (n + NT - 1) / NT;
    augment_kernel<<<(unsigned)(g > 65536 ? 65536 : g), NT, 0, as_stream(stream)>>>(B, S, (const uint8_t*)img,
                                                                                  (const uint8_t*)mask, params, out_img,
                                                                                  out_mask);
    return check_launch("augment_batch");
}
