// Diagnostic (not product code): does gfx950 apply VOP3P neg_lo/neg_hi to
// 16-bit integer operands (v_pk_max_i16 x, -x = |x|; v_pk_add_u16 x, -y)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t *in, uint32_t *out)
{
    const uint32_t x = in[threadIdx.x], y = in[threadIdx.x + 64];
    uint32_t r0, r1, r2, r3;
    asm volatile("v_pk_max_i16 %0, %1, %1 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r0) : "v"(x));
    asm volatile("v_pk_add_u16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r1) : "v"(x), "v"(y));
    asm volatile("v_pk_sub_i16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r2) : "v"(x), "v"(y));
    asm volatile("v_pk_add_i16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r3) : "v"(x), "v"(y));
    out[4 * threadIdx.x] = r0;
    out[4 * threadIdx.x + 1] = r1;
    out[4 * threadIdx.x + 2] = r2;
    out[4 * threadIdx.x + 3] = r3;
}
int main()
{
    uint32_t h[128], o[256];
    for (int i = 0; i < 64; i++) {
        const int16_t lo = int16_t(i * 37 - 1000), hi = int16_t(500 - i * 23);
        h[i] = uint16_t(lo) | uint32_t(uint16_t(hi)) << 16;
        h[i + 64] = uint32_t(uint16_t(i * 3)) | uint32_t(uint16_t(i * 5)) << 16;
    }
    uint32_t *din, *dout;
    hipMalloc(&din, sizeof(h));
    hipMalloc(&dout, sizeof(o));
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
    hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    int ok_abs = 1, ok_add = 1, ok_sub = 1, ok_addi = 1;
    for (int i = 0; i < 64; i++) {
        const int16_t xl = int16_t(h[i]), xh = int16_t(h[i] >> 16), yl = int16_t(h[i + 64]), yh = int16_t(h[i + 64] >> 16);
        auto pk = [](int a, int b) { return uint32_t(uint16_t(a)) | uint32_t(uint16_t(b)) << 16; };
        if (o[4 * i] != pk(abs(xl), abs(xh))) ok_abs = 0;
        if (o[4 * i + 1] != pk(xl - yl, xh - yh)) ok_add = 0;
        if (o[4 * i + 2] != pk(xl + yl, xh + yh)) ok_sub = 0;
        if (o[4 * i + 3] != pk(xl - yl, xh - yh)) ok_addi = 0;
        if (i < 3) printf("x=%08x y=%08x max(x,-x)=%08x add_u16(x,-y)=%08x sub_i16(x,-y)=%08x add_i16(x,-y)=%08x\n", h[i], h[i + 64], o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
    }
    printf("neg honoured: pk_max_i16 abs %d, pk_add_u16 %d, pk_sub_i16 %d, pk_add_i16 %d\n", ok_abs, ok_add, ok_sub, ok_addi);
    return 0;
}
