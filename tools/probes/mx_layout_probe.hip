// Probe 2: which operand bytes does each lane's E8M0 scale of v_mfma_scale_f32_32x32x64_f8f6f4 apply to,
// and which (lane, byte) of B pairs with a (lane, byte) of A.  A = one nonzero byte (1.0 e4m3 = 0x38)
// at lane (row 0, half H) byte J; scale_a = 127 for lanes h = 0, 128 (2.0) for lanes h = 1.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// mode 0: B all 1.0 (scale 127) -> D[0][*] = scale that hit A's byte
// mode 1: B has a single 1.0 at lane (col 0, half HB) byte JB -> D[0][0] != 0 iff paired
__global__ void k(float* out, int H, int J, int mode, int HB, int JB) {
    const int lane = threadIdx.x;
    const int r = lane & 31, h = lane >> 5;
    i32x8 a = {}, b = {};
    unsigned char* pa = (unsigned char*)&a;
    unsigned char* pb = (unsigned char*)&b;
    if (r == 0 && h == H) pa[J] = 0x38;
    for (int j = 0; j < 32; ++j) pb[j] = mode == 0 ? 0x38 : ((r == 0 && h == HB && j == JB) ? 0x38 : 0);
    const int sa = 127 + h;
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 127);
    out[lane] = c[0];   // D[row (i&3)+8(i>>2)+4h][col r]: i = 0, h = 0 -> D[0][r]
}

int main() {
    float* d;
    hipMalloc(&d, 64 * 4);
    float hb[64];
    printf("scale association (A byte at lane half H, byte J; lane-half scales 1 / 2):\n");
    for (int H = 0; H < 2; ++H)
        for (int J : {0, 7, 8, 15, 16, 23, 24, 31}) {
            k<<<1, 64>>>(d, H, J, 0, 0, 0);
            hipMemcpy(hb, d, sizeof(hb), hipMemcpyDeviceToHost);
            printf("  H=%d J=%2d -> D[0][0]=%g\n", H, J, hb[0]);
        }
    printf("pairing (A lane half H byte J with B lane half HB byte JB):\n");
    for (int H = 0; H < 2; ++H)
        for (int J : {0, 5, 16, 31}) {
            int found = 0;
            for (int HB = 0; HB < 2; ++HB)
                for (int JB = 0; JB < 32; ++JB) {
                    k<<<1, 64>>>(d, H, J, 1, HB, JB);
                    hipMemcpy(hb, d, sizeof(hb), hipMemcpyDeviceToHost);
                    if (hb[0] != 0.f) { printf("  A(H=%d,J=%2d) pairs B(H=%d,J=%2d) value %g\n", H, J, HB, JB, hb[0]); found = 1; }
                }
            if (!found) printf("  A(H=%d,J=%2d) pairs nothing\n", H, J);
        }
    hipFree(d);
    return 0;
}
