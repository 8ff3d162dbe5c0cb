// FETCH_SIZE calibration for the paired-row PNG kernel's input loads
// (png_pair_kernels.hip, load_group): the same 64 x 4K tc8 filtered stream
// (4096 rows of 1 + 12288 bytes per image), read in the kernel's shape -- a
// wave per 128-row band, lane j holding rows 2j and 2j+1, one group of 8
// 12-byte chunks per row per step of the loop (six 16-byte loads and one
// dword at the row's dword-aligned offset, 96 bytes apart from one group to
// the next) -- with no arithmetic.  The known byte count is the stream
// itself; rocprofv3 --pmc FETCH_SIZE of this launch divided by it is the
// counter's factor for this access shape (MI355X_MICROARCH.md: calibrate an
// access width before trusting an absolute).  mode 1 reads the same bytes
// as 16 bytes per lane, fully linear (the guide's calibrated case); mode 2
// reads each band cooperatively: 8 lanes per row, 128 contiguous bytes, 8
// rows per instruction, rows walked in 128-byte steps (the shape a
// line-staged input would have).
// Usage: png_load_pattern <mode 0|1|2|3|5|6|7> [waves per CU, modes 0/2/3/5/6/7; default 8]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kImages = 64, kW = 4096, kH = 4096;
constexpr size_t kRow = 1 + size_t(kW) * 3;   // filter byte + RGB
constexpr size_t kImg = kRow * kH;             // 50,335,744 B
constexpr int kBands = kH / 128;

__global__ __launch_bounds__(64) void band_loads(const unsigned char *__restrict__ in, unsigned *__restrict__ sink,
                                                 unsigned mask)
{
    const int lane = threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
    for (int b = blockIdx.x; b < kImages * kBands; b += gridDim.x) {
        const int img = b / kBands, band = b % kBands;
        const unsigned char *band0 = in + size_t(img) * kImg + size_t(band) * 128 * kRow;
        const uintptr_t a0 = reinterpret_cast<uintptr_t>(band0) & ~uintptr_t(3);
        const unsigned delta = static_cast<unsigned>(reinterpret_cast<uintptr_t>(band0) - a0);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(a0), 0, 0x7ffffff0, 0x00020000);
        const unsigned r0 = delta + unsigned(2 * lane) * unsigned(kRow), r1 = r0 + unsigned(kRow);
        const unsigned d0 = (r0 + 1) & ~3u, d1 = (r1 + 1) & ~3u;
        for (int g = 0; g < kW * 3 / 96 + 1; g++) {
#pragma unroll
            for (int i = 0; i < 6; i++) {
                acc ^= __builtin_amdgcn_raw_buffer_load_b128(rsrc, d0 + 96 * g + 16 * i, 0, 0);
                acc ^= __builtin_amdgcn_raw_buffer_load_b128(rsrc, d1 + 96 * g + 16 * i, 0, 0);
            }
            acc[0] ^= __builtin_amdgcn_raw_buffer_load_b32(rsrc, d0 + 96 * g + 96, 0, 0);
            acc[1] ^= __builtin_amdgcn_raw_buffer_load_b32(rsrc, d1 + 96 * g + 96, 0, 0);
        }
    }
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) & mask) sink[blockIdx.x * 64 + lane] = acc[0];
}

__global__ __launch_bounds__(64) void coop_loads(const unsigned char *__restrict__ in, unsigned *__restrict__ sink,
                                                 unsigned mask)
{
    const int lane = threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
    for (int b = blockIdx.x; b < kImages * kBands; b += gridDim.x) {
        const int img = b / kBands, band = b % kBands;
        const unsigned char *band0 = in + size_t(img) * kImg + size_t(band) * 128 * kRow;
        const uintptr_t a0 = reinterpret_cast<uintptr_t>(band0) & ~uintptr_t(127);
        const unsigned delta = static_cast<unsigned>(reinterpret_cast<uintptr_t>(band0) - a0);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(a0), 0, 0x7ffffff0, 0x00020000);
        for (int g = 0; g < int(kRow / 128) + 1; g++) {
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const unsigned row = 8 * i + lane / 8;
                const unsigned off = ((delta + row * unsigned(kRow)) & ~127u) + 128 * g + 16 * (lane % 8);
                acc ^= __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
            }
        }
    }
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) & mask) sink[blockIdx.x * 64 + lane] = acc[0];
}

// mode 3: the STREAM instance's loads (png_pair_kernels.hip, load_units):
// per group of 8 12-byte chunks and per row half h (rows 2j + h), six
// instructions whose lane-piece n = 64 i + lane is piece n % 6 of row
// 2 (n / 6) + h's 96-byte window -- unaligned 16-byte loads, a row's window
// on 6 consecutive lanes -- one group after the other.  mode 5: the same
// instruction shape, but only group `first` of every row (each row's window
// read once): the fetch granularity of this shape, by comparing FETCH_SIZE
// with the 64-byte sectors and 128-byte lines the windows cover (printed).
// mode 6 / 7: mode 3 with every offset rounded down to 16 / 4 bytes (the
// same rows and lines per instruction, aligned lane accesses).
__global__ __launch_bounds__(64) void stream_units(const unsigned char *__restrict__ in, unsigned *__restrict__ sink,
                                                   unsigned mask, int once, unsigned align_mask)
{
    const int lane = threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
    for (int b = blockIdx.x; b < kImages * kBands; b += gridDim.x) {
        const int img = b / kBands, band = b % kBands;
        const unsigned char *band0 = in + size_t(img) * kImg + size_t(band) * 128 * kRow;
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(band0), 0, 0x7ffffff0, 0x00020000);
        unsigned voff[2][6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const int n = 64 * i + lane;
            voff[0][i] = (unsigned(2 * (n / 6)) * unsigned(kRow) + 1u + 16u * unsigned(n % 6)) & align_mask;
            voff[1][i] = (voff[0][i] + unsigned(kRow)) & align_mask;
        }
        const int ng = once ? 1 : kW * 3 / 96;
        for (int g = 0; g < ng; g++) {
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int i = 0; i < 6; i++)
                    acc ^= __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff[h][i] + 96u * unsigned(g), 0, 0);
        }
    }
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) & mask) sink[blockIdx.x * 64 + lane] = acc[0];
}

// mode 8: two groups' windows of a row in one unit -- 192 contiguous bytes
// a row on 12 consecutive lanes, ~5.3 rows an instruction -- every second
// group, for row quarters (the shape of a 2-group stream unit).
__global__ __launch_bounds__(64) void stream_units2(const unsigned char *__restrict__ in, unsigned *__restrict__ sink,
                                                    unsigned mask)
{
    const int lane = threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
    for (int b = blockIdx.x; b < kImages * kBands; b += gridDim.x) {
        const int img = b / kBands, band = b % kBands;
        const unsigned char *band0 = in + size_t(img) * kImg + size_t(band) * 128 * kRow;
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char *>(band0), 0, 0x7ffffff0, 0x00020000);
        unsigned voff[4][6];
#pragma unroll
        for (int q = 0; q < 4; q++) // row quarter q: rows 4 r + q, r < 32
#pragma unroll
            for (int i = 0; i < 6; i++) {
                const int n = 64 * i + lane; // 384 lane-pieces: row n / 12, piece n % 12
                voff[q][i] = unsigned(4 * (n / 12) + q) * unsigned(kRow) + 1u + 16u * unsigned(n % 12);
            }
        for (int g = 0; g < kW * 3 / 96; g += 2) {
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int i = 0; i < 6; i++)
                    acc ^= __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff[q][i] + 96u * unsigned(g), 0, 0);
        }
    }
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) & mask) sink[blockIdx.x * 64 + lane] = acc[0];
}

__global__ __launch_bounds__(256) void linear_loads(const u32x4 *__restrict__ in, size_t n, unsigned *__restrict__ sink,
                                                    unsigned mask)
{
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) acc ^= in[i];
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) & mask) sink[threadIdx.x] = acc[0];
}

int main(int argc, char **argv)
{
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const int wpc = argc > 2 ? atoi(argv[2]) : 8;
    const size_t bytes = kImg * kImages + 4096;
    unsigned char *in = nullptr;
    unsigned *sink = nullptr;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&sink, 1 << 24) != hipSuccess) return 1;
    (void)hipMemset(in, 1, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int it = 0; it < 5; it++) {
        (void)hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(band_loads, dim3(256 * wpc), dim3(64), 0, 0, in, sink, 0u);
        else if (mode == 2) hipLaunchKernelGGL(coop_loads, dim3(256 * wpc), dim3(64), 0, 0, in, sink, 0u);
        else if (mode == 8) hipLaunchKernelGGL(stream_units2, dim3(256 * wpc), dim3(64), 0, 0, in, sink, 0u);
        else if (mode == 3 || mode == 5 || mode == 6 || mode == 7)
            hipLaunchKernelGGL(stream_units, dim3(256 * wpc), dim3(64), 0, 0, in, sink, 0u, mode == 5 ? 1 : 0,
                               mode == 6 ? ~15u : mode == 7 ? ~3u : ~0u);
        else hipLaunchKernelGGL(linear_loads, dim3(8192), dim3(256), 0, 0, reinterpret_cast<const u32x4 *>(in),
                                 kImg * kImages / 16, sink, 0u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    if (mode == 5) { // the sectors / lines the windows cover (the buffer's base is 256-byte aligned)
        size_t sectors = 0, lines = 0, bytes = 0;
        for (int b = 0; b < kImages * kBands; b++)
            for (int r = 0; r < 128; r++) {
                const size_t a = size_t(b / kBands) * kImg + size_t(b % kBands) * 128 * kRow + size_t(r) * kRow + 1;
                sectors += (a + 95) / 64 - a / 64 + 1;
                lines += (a + 95) / 128 - a / 128 + 1;
                bytes += 96;
            }
        printf("mode 5: %.3f ms; windows %zu B, 64-B sectors %zu (%zu B), 128-B lines %zu (%zu B)\n", best, bytes,
               sectors, sectors * 64, lines, lines * 128);
        return 0;
    }
    printf("mode %d, %d waves/CU: %.3f ms, %zu true bytes, %.1f GB/s\n", mode, wpc, best, kImg * kImages,
           kImg * kImages / (best * 1e-3) / 1e9);
    return 0;
}
