// pool_trim_copy.hip -- library-free check of the sequence behind the lost
// leaf upload (DESIGN.md §2 "Device memory"): stream-ordered allocations on a
// non-blocking stream, kernels writing them, frees, a device-wide sync and
// hipMemPoolTrimTo(pool, 0), then a fresh hipMallocAsync on the null stream
// (synchronised, as dx_malloc does) filled from a pinned host buffer on the
// non-blocking stream and read back.  Prints the number of lost copies.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/pool_trim_copy tools/micro/pool_trim_copy.hip
// usage: pool_trim_copy [rounds=200] [trim=1] [threshold_max=1]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void fill(uint64_t* p, size_t n, uint64_t salt)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (i * 0x9E3779B97F4A7C15ull) ^ salt;
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 200;
    const bool trim = argc > 2 ? std::atoi(argv[2]) != 0 : true;
    const bool keep = argc > 3 ? std::atoi(argv[3]) != 0 : true;
    CK(hipSetDevice(0));
    hipMemPool_t pool;
    CK(hipDeviceGetDefaultMemPool(&pool, 0));
    if (keep) {  // the library's setting: freed memory stays in the pool
        uint64_t t = UINT64_MAX;
        CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &t));
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t max_n = 8u << 20;  // up to 64 MiB per block
    uint64_t *stage = nullptr, *back = nullptr;
    CK(hipHostMalloc((void**)&stage, max_n * 8, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&back, max_n * 8, hipHostMallocDefault));
    uint64_t rng = 12345;
    auto next = [&rng]() {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        return rng;
    };
    int lost = 0;
    for (int r = 0; r < rounds; r++) {
        // a "grid": blocks of many sizes, written by kernels, then freed
        std::vector<uint64_t*> blocks;
        for (int k = 0; k < 24; k++) {
            const size_t n = 64 + next() % max_n;
            uint64_t* p = nullptr;
            CK(hipMallocAsync((void**)&p, n * 8, s));
            hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, s, p, n, (uint64_t)r);
            blocks.push_back(p);
        }
        for (uint64_t* p : blocks) CK(hipFreeAsync(p, s));
        CK(hipDeviceSynchronize());
        if (trim) CK(hipMemPoolTrimTo(pool, 0));
        // the next grid's first upload
        const size_t n = 64 + next() % max_n;
        uint64_t* d = nullptr;
        CK(hipMallocAsync((void**)&d, n * 8, nullptr));
        CK(hipStreamSynchronize(nullptr));
        for (size_t i = 0; i < n; i++) stage[i] = i * 2654435761ull + (uint64_t)r;
        CK(hipMemcpyAsync(d, stage, n * 8, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        std::memset(back, 0, n * 8);
        CK(hipMemcpyAsync(back, d, n * 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        size_t bad = 0;
        for (size_t i = 0; i < n; i++) bad += back[i] != stage[i];
        if (bad) {
            lost++;
            std::printf("round %d: %zu of %zu words differ\n", r, bad, n);
        }
        CK(hipFreeAsync(d, nullptr));
        CK(hipDeviceSynchronize());
    }
    std::printf("pool_trim_copy rounds=%d trim=%d threshold_max=%d lost=%d\n", rounds, trim, keep, lost);
    CK(hipHostFree(stage));
    CK(hipHostFree(back));
    CK(hipStreamDestroy(s));
    return lost ? 1 : 0;
}
