// Memory-pattern floor of the fused JPEG kernel's launch (64 x 4K 4:2:0):
// 1.61 GB of coefficient reads + 4.29 GB of RGBA writes, no arithmetic.
//   mode 0 "task":   the block kernel's task shape -- per task 8 KiB of Y grid
//                    (2 block rows x 4 KiB), 2 KiB Cb, 2 KiB Cr, then 16 output
//                    rows x 2 KiB at the image's 16 KiB row stride
//   mode 1 "linear": per task 12 KiB read and 32 KiB written, both contiguous
//   mode 2 "write":  mode 0's stores only
//   mode 3 "task4k": tasks twice as wide (4 KiB row segments, 8 output rows)
//   mode 4 "spread": mode 0 with VALU work (argv[5] x 64 multiply-adds)
//                    before each row's two stores
//   mode 5 "burst":  mode 4's VALU work, then all 32 stores together
// Usage: mem_pattern <mode> <waves_per_cu> <nt 0|1> [xcd_remap 0|1]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kFrames = 64, kW = 4096, kH = 4096;
constexpr size_t kRgba = size_t(kW) * kH * 4, kYGrid = size_t(kW) * kH, kCGrid = kYGrid / 4;

template <int MODE, int NT>
__global__ __launch_bounds__(64) void pattern(const unsigned char *__restrict__ coef, unsigned char *__restrict__ out,
                                               int total_tasks, unsigned sink_mask, int remap, int work)
{
    const int lane = threadIdx.x;
    int t0 = blockIdx.x;
    if (remap) { // consecutive tasks on one XCD (the block kernel's ZPX_JPEGB_XCD_REMAP)
        const int nw = static_cast<int>(gridDim.x), w = static_cast<int>(blockIdx.x);
        const int q = nw / 8, r = nw % 8, x = w % 8;
        t0 = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8;
    }
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7ffffff0, 0x00020000);
    u32x4 acc = {0, 0, 0, 0};
    for (int t = t0; t < total_tasks; t += gridDim.x) {
        if constexpr (MODE == 0 || MODE == 2 || MODE == 3 || MODE == 4 || MODE == 5) {
            constexpr int TW = MODE == 3 ? 2 : 1;          // task width in 2 KiB row segments
            constexpr int ROWS = MODE == 3 ? 8 : 16;       // output rows per task
            const int tasks_x = 8 / TW, per_frame = tasks_x * (kH / ROWS);
            const int f = t / per_frame, r = t - f * per_frame, row = r / tasks_x, tx = r - row * tasks_x;
            if constexpr (MODE != 2) {
                const unsigned char *y = coef + f * (kYGrid + 2 * kCGrid);
                const unsigned char *cb = y + kYGrid, *cr = cb + kCGrid;
                const size_t yrow = size_t(row) * (ROWS / 8) * 512 * 64; // block rows of 512 blocks
#pragma unroll
                for (int i = 0; i < 4 * TW * (ROWS / 8); i++) {
                    const int br = i / (4 * TW), piece = i % (4 * TW);
                    acc ^= *reinterpret_cast<const u32x4 *>(y + yrow + size_t(br) * 32768 + tx * 4096 * TW + piece * 1024 + 16 * lane);
                }
                const size_t crow = size_t(row) * (ROWS / 16) * 256 * 64;
                const int cpieces = MODE == 3 ? 1 : 2; // MODE 3: 8 rows = half a chroma block row
#pragma unroll
                for (int i = 0; i < cpieces * TW; i++) {
                    acc ^= *reinterpret_cast<const u32x4 *>(cb + crow + tx * 2048 * TW + i * 1024 + 16 * lane);
                    acc ^= *reinterpret_cast<const u32x4 *>(cr + crow + tx * 2048 * TW + i * 1024 + 16 * lane);
                }
            }
            unsigned char *o = out + f * kRgba + size_t(row) * ROWS * kW * 4 + size_t(tx) * 2048 * TW;
            const uint64_t ob = reinterpret_cast<uint64_t>(o);
            const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(
                (uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(ob >> 32)) << 32 | (unsigned)__builtin_amdgcn_readfirstlane((unsigned)ob)),
                0, 0x7ffffff0, 0x00020000);
            u32x4 v = acc & sink_mask;
            auto burn = [&]() {
                // `work` x 64 independent multiply-adds (four chains), ~the fused kernel's VALU per row
                unsigned a0 = v[0] | 1, a1 = v[1] | 3, a2 = v[2] | 5, a3 = v[3] | 7;
                for (int i = 0; i < work; i++) {
#pragma unroll
                    for (int k = 0; k < 16; k++) {
                        a0 = __mul24(a0, 0x10101) + a1;
                        a1 = __mul24(a1, 0x10101) + a2;
                        a2 = __mul24(a2, 0x10101) + a3;
                        a3 = __mul24(a3, 0x10101) + a0;
                    }
                }
                v[0] ^= (a0 ^ a1 ^ a2 ^ a3) & sink_mask;
            };
            if constexpr (MODE == 5)
                for (int rr = 0; rr < ROWS; rr++) burn();
#pragma unroll
            for (int rr = 0; rr < ROWS; rr++) {
                if constexpr (MODE == 4) burn();
#pragma unroll
                for (int h = 0; h < 2 * TW; h++)
                    __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, rr * kW * 4 + h * 1024 + 16 * lane, 0, NT ? 2 : 0);
            }
        } else {
            const unsigned char *c = coef + size_t(t) * 12288;
#pragma unroll
            for (int i = 0; i < 12; i++) acc ^= *reinterpret_cast<const u32x4 *>(c + i * 1024 + 16 * lane);
            const u32x4 v = acc & sink_mask;
            (void)rsrc;
            unsigned char *o = out + size_t(t) * 32768;
            const uint64_t ob = reinterpret_cast<uint64_t>(o);
            const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(
                (uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(ob >> 32)) << 32 | (unsigned)__builtin_amdgcn_readfirstlane((unsigned)ob)),
                0, 0x7ffffff0, 0x00020000);
#pragma unroll
            for (int h = 0; h < 32; h++) __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, h * 1024 + 16 * lane, 0, NT ? 2 : 0);
        }
    }
}

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                                   \
            return 1;                                                                                                  \
        }                                                                                                              \
    } while (0)

template <int MODE, int NT>
void launch(int grid, const unsigned char *c, unsigned char *o, int tasks, int remap, int work)
{
    hipLaunchKernelGGL((pattern<MODE, NT>), dim3(grid), dim3(64), 0, 0, c, o, tasks, 0u, remap, work);
}

int main(int argc, char **argv)
{
    const int mode = argc > 1 ? atoi(argv[1]) : 0, wpc = argc > 2 ? atoi(argv[2]) : 12, nt = argc > 3 ? atoi(argv[3]) : 1;
    const int remap = argc > 4 ? atoi(argv[4]) : 0, work = argc > 5 ? atoi(argv[5]) : 4;
    const size_t cbytes = size_t(kFrames) * (kYGrid + 2 * kCGrid), obytes = size_t(kFrames) * kRgba;
    unsigned char *c = nullptr, *o = nullptr;
    CK(hipMalloc(&c, cbytes));
    CK(hipMalloc(&o, obytes));
    CK(hipMemset(c, 1, cbytes));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int tasks = mode == 3 ? kFrames * 4 * (kH / 8) : kFrames * 8 * (kH / 16);
    const int grid = cus * wpc;
    auto run = [&]() {
        switch (mode * 2 + (nt ? 1 : 0)) {
        case 0: launch<0, 0>(grid, c, o, tasks, remap, work); break;
        case 1: launch<0, 1>(grid, c, o, tasks, remap, work); break;
        case 2: launch<1, 0>(grid, c, o, tasks, remap, work); break;
        case 3: launch<1, 1>(grid, c, o, tasks, remap, work); break;
        case 4: launch<2, 0>(grid, c, o, tasks, remap, work); break;
        case 5: launch<2, 1>(grid, c, o, tasks, remap, work); break;
        case 6: launch<3, 0>(grid, c, o, tasks, remap, work); break;
        case 7: launch<3, 1>(grid, c, o, tasks, remap, work); break;
        case 8: launch<4, 0>(grid, c, o, tasks, remap, work); break;
        case 9: launch<4, 1>(grid, c, o, tasks, remap, work); break;
        case 10: launch<5, 0>(grid, c, o, tasks, remap, work); break;
        case 11: launch<5, 1>(grid, c, o, tasks, remap, work); break;
        }
    };
    for (int i = 0; i < 3; i++) run();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int iters = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; i++) run();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= iters;
    const double bytes = double(obytes) + (mode == 2 ? 0.0 : double(cbytes));
    printf("mode %d wpc %d nt %d remap %d work %d: %.4f ms/launch, %.1f GB/s (%.3f of 8 TB/s)\n", mode, wpc, nt, remap, work, ms, bytes / ms / 1e6,
           bytes / ms / 1e6 / 8000.0);
    return 0;
}
