// launch_chain.hip -- what a chain of small dependent kernels costs on one
// stream (the adaptive step is ~100 of them): per-kernel time of K tiny
// launches back to back, of the same K captured once in a HIP graph and
// replayed, and of K launches each followed by a small device->host read
// (hipMemcpyAsync + hipStreamSynchronize every `sync_every` kernels).
// build: hipcc --offload-arch=gfx950 -O3 -o launch_chain launch_chain.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__global__ void k_touch(unsigned* p, unsigned n)
{
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1u;
}

int main(int argc, char** argv)
{
    const int K = argc > 1 ? std::atoi(argv[1]) : 100;
    const unsigned n = argc > 2 ? (unsigned)std::atoi(argv[2]) : 218000;  // elements per kernel
    unsigned* d = nullptr;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemset(d, 0, n * 4));
    unsigned* h = nullptr;
    CK(hipHostMalloc(&h, 64, hipHostMallocDefault));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const dim3 g((n + 255) / 256), b(256);
    auto chain = [&] {
        for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_touch, g, b, 0, st, d, n);
    };
    for (int w = 0; w < 3; w++) chain();
    CK(hipStreamSynchronize(st));
    const int R = 20;
    // plain chain
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < R; r++) chain();
    CK(hipStreamSynchronize(st));
    auto t1 = std::chrono::steady_clock::now();
    const double plain = std::chrono::duration<double, std::micro>(t1 - t0).count() / (R * K);
    // graph
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    chain();
    CK(hipStreamEndCapture(st, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < R; r++) CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    t1 = std::chrono::steady_clock::now();
    const double graph = std::chrono::duration<double, std::micro>(t1 - t0).count() / (R * K);
    // chain with a read-back every few kernels
    std::printf("K=%d n=%u: plain %.2f us/kernel, graph %.2f us/kernel\n", K, n, plain, graph);
    for (int every : {1, 5, 10, 25}) {
        t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < R; r++)
            for (int k = 0; k < K; k++) {
                hipLaunchKernelGGL(k_touch, g, b, 0, st, d, n);
                if ((k + 1) % every == 0) {
                    CK(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, st));
                    CK(hipStreamSynchronize(st));
                }
            }
        CK(hipStreamSynchronize(st));
        t1 = std::chrono::steady_clock::now();
        std::printf("  read-back every %2d kernels: %.2f us/kernel\n", every,
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / (R * K));
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gr));
    CK(hipFree(d));
    CK(hipHostFree(h));
    return 0;
}
