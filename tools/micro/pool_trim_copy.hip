// pool_trim_copy.hip -- library-free check of the sequence behind the lost
// leaf upload (DESIGN.md §2 "Device memory"): stream-ordered allocations on a
// non-blocking stream written by kernels and freed, optionally
// hipMemPoolTrimTo(pool, 0), then a fresh block filled (pinned-host copy or
// kernel) on the non-blocking stream and checked twice: on the device (a
// kernel counts wrong words) and on the host after a copy back.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/pool_trim_copy tools/micro/pool_trim_copy.hip
// usage: pool_trim_copy rounds trim threshold_max alloc kernel_fill churn
//   alloc: 0 hipMallocAsync on the null stream, 1 on the copying stream,
//          2 hipMalloc (no pool)
//   kernel_fill: the fresh block is written by a kernel instead of the copy
//   churn: 0 no other allocations (only the checked block), 1 the 24 blocks
//          (hipMallocAsync / hipFreeAsync), 2 the 24 blocks with hipMalloc / hipFree
// exit 0 either way; the last line reports the rounds whose data was wrong
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                          \
        }                                                                                          \
    } while (0)

__device__ __host__ inline uint64_t pattern(uint64_t i, uint64_t salt) { return (i * 0x9E3779B97F4A7C15ull) ^ salt; }

__global__ void fill(uint64_t* p, size_t n, uint64_t salt)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = pattern(i, salt);
}

__global__ void verify(const uint64_t* p, size_t n, uint64_t salt, unsigned long long* bad)
{
    unsigned long long b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != pattern(i, salt);
    if (b) atomicAdd(bad, b);
}

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 100;
    const bool trim = argc > 2 && std::atoi(argv[2]);
    const bool keep = argc > 3 ? std::atoi(argv[3]) != 0 : true;
    const int alloc = argc > 4 ? std::atoi(argv[4]) : 0;
    const bool kfill = argc > 5 && std::atoi(argv[5]);
    const int churn = argc > 6 ? std::atoi(argv[6]) : 1;
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
    unsigned long long* d_bad = nullptr;
    CK(hipMalloc((void**)&d_bad, 8));
    uint64_t rng = 12345;
    auto next = [&rng]() {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        return rng;
    };
    int lost_dev = 0, lost_host = 0;
    for (int r = 0; r < rounds; r++) {
        if (churn) {  // a "grid": blocks of many sizes, written by kernels, then freed
            std::vector<uint64_t*> blocks;
            for (int k = 0; k < 24; k++) {
                const size_t n = 64 + next() % (max_n - 64);
                uint64_t* p = nullptr;
                if (churn == 2) CK(hipMalloc((void**)&p, n * 8));
                else CK(hipMallocAsync((void**)&p, n * 8, s));
                hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, s, p, n, (uint64_t)r);
                CK(hipGetLastError());
                blocks.push_back(p);
            }
            if (churn == 2) CK(hipDeviceSynchronize());
            for (uint64_t* p : blocks) {
                if (churn == 2) CK(hipFree(p));
                else CK(hipFreeAsync(p, s));
            }
        }
        CK(hipDeviceSynchronize());
        if (trim) CK(hipMemPoolTrimTo(pool, 0));
        const size_t n = 64 + next() % (max_n - 64);
        const uint64_t salt = 1000000 + (uint64_t)r;
        uint64_t* d = nullptr;
        if (alloc == 2) CK(hipMalloc((void**)&d, n * 8));
        else CK(hipMallocAsync((void**)&d, n * 8, alloc == 1 ? s : nullptr));
        CK(hipDeviceSynchronize());
        if (kfill) {
            hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, s, d, n, salt);
            CK(hipGetLastError());
        } else {
            for (size_t i = 0; i < n; i++) stage[i] = pattern(i, salt);
            CK(hipMemcpyAsync(d, stage, n * 8, hipMemcpyHostToDevice, s));
        }
        CK(hipMemsetAsync(d_bad, 0, 8, s));
        hipLaunchKernelGGL(verify, dim3(256), dim3(256), 0, s, (const uint64_t*)d, n, salt, d_bad);
        CK(hipGetLastError());
        unsigned long long bad_dev = 0;
        CK(hipMemcpyAsync(&bad_dev, d_bad, 8, hipMemcpyDeviceToHost, s));
        std::memset(back, 0xab, n * 8);
        CK(hipMemcpyAsync(back, d, n * 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        size_t bad = 0, first = n;
        for (size_t i = 0; i < n; i++)
            if (back[i] != pattern(i, salt)) {
                bad++;
                if (first == n) first = i;
            }
        lost_dev += bad_dev != 0;
        lost_host += bad != 0;
        if ((bad || bad_dev) && lost_host + lost_dev <= 6)
            std::printf("round %d: device check %llu, host check %zu of %zu words wrong, first at %zu (%016llx)\n", r,
                        bad_dev, bad, n, first, first < n ? (unsigned long long)back[first] : 0ull);
        if (alloc == 2) CK(hipFree(d));
        else CK(hipFreeAsync(d, s));
        CK(hipDeviceSynchronize());
    }
    std::printf("pool_trim_copy rounds=%d trim=%d threshold_max=%d alloc=%d kernel_fill=%d churn=%d "
                "wrong_on_device=%d wrong_on_host=%d\n",
                rounds, trim, keep, alloc, kfill, churn, lost_dev, lost_host);
    CK(hipHostFree(stage));
    CK(hipHostFree(back));
    CK(hipFree(d_bad));
    CK(hipStreamDestroy(s));
    return 0;
}
