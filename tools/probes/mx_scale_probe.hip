// Probe: semantics of the scale operands of v_mfma_scale_f32_32x32x64_f8f6f4 on gfx950
// (E8M0 encoding, per-lane granularity).  A = B = 1.0 (e4m3 0x38) everywhere, K = 64.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ void k(float* out, int sa_base, int sb_base) {
    const int lane = threadIdx.x;
    const int r = lane & 31, h = lane >> 5;
    i32x8 a, b;
    for (int i = 0; i < 8; ++i) { a[i] = 0x38383838; b[i] = 0x38383838; }
    int sa = sa_base, sb = sb_base;
    if (MODE == 1) sa = sa_base + h;            // per lane half of A
    if (MODE == 2) sa = sa_base + (r == 3);     // A row 3
    if (MODE == 3) sb = sb_base + (r == 5);     // B column 5
    if (MODE == 4) sb = sb_base + h;            // per lane half of B
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
    for (int i = 0; i < 16; ++i) out[lane * 16 + i] = c[i];
}

int main() {
    float* d;
    hipMalloc(&d, 64 * 16 * 4);
    float hbuf[64 * 16];
    auto run = [&](auto kern, int sa, int sb, const char* tag) {
        kern<<<1, 64>>>(d, sa, sb);
        hipMemcpy(hbuf, d, sizeof(hbuf), hipMemcpyDeviceToHost);
        // D[row][col]: col = lane & 31, row = (i&3) + 8*(i>>2) + 4*(lane>>5)
        printf("%s sa=%d sb=%d: D[0][0]=%g D[3][0]=%g D[0][5]=%g D[4][0]=%g\n", tag, sa, sb, hbuf[0], hbuf[3 * 16 / 16 * 0 + 3],
               hbuf[5 * 16], hbuf[32 * 16 + 0]);
    };
    run(k<0>, 0, 0, "uniform");
    run(k<0>, 127, 127, "uniform");
    run(k<0>, 128, 127, "uniform");
    run(k<0>, 127, 126, "uniform");
    run(k<1>, 127, 127, "A by lane half");
    run(k<2>, 127, 127, "A row 3");
    run(k<3>, 127, 127, "B col 5");
    run(k<4>, 127, 127, "B by lane half");
    hipFree(d);
    return 0;
}
