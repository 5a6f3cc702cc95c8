// cub_host_cost.hip -- host-side cost of the hipcub calls the adaptive step
// uses (DeviceSelect::Flagged / Unique, DeviceRadixSort::SortKeys), without
// synchronising: the time until each call returns, per call, at the sizes
// of configs[2]'s step.
//   hipcc --offload-arch=gfx950 -O2 -o cub_host_cost cub_host_cost.hip && ./cub_host_cost
#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                              \
        }                                                                          \
    } while (0)

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int N = 1 << 20;
    uint64_t *keys, *out;
    uint8_t* flags;
    uint64_t* cnt;
    CK(hipMalloc(&keys, N * 8));
    CK(hipMalloc(&out, N * 8));
    CK(hipMalloc(&flags, N));
    CK(hipMalloc(&cnt, 16));
    CK(hipMemset(flags, 1, N));
    std::vector<uint64_t> h(N);
    for (int i = 0; i < N; i++) h[i] = (uint64_t)(i * 2654435761u) % 5000000;
    CK(hipMemcpy(keys, h.data(), N * 8, hipMemcpyHostToDevice));
    void* tmp = nullptr;
    size_t tb = 64 << 20;
    CK(hipMalloc(&tmp, tb));
    for (int n : {20000, 60000, 220000}) {
        for (int bits : {23, 64}) {
            double t_sort = 0, t_sel = 0, t_uni = 0;
            const int reps = 20;
            for (int r = 0; r < reps + 2; r++) {
                size_t b = tb;
                double t0 = now_us();
                CK(hipcub::DeviceSelect::Flagged(tmp, b, keys, flags, out, cnt, n, st));
                double t1 = now_us();
                b = tb;
                CK(hipcub::DeviceRadixSort::SortKeys(tmp, b, keys, out, n, 0, bits, st));
                double t2 = now_us();
                b = tb;
                CK(hipcub::DeviceSelect::Unique(tmp, b, out, keys, cnt + 1, n, st));
                double t3 = now_us();
                CK(hipStreamSynchronize(st));
                CK(hipMemcpy(keys, h.data(), N * 8, hipMemcpyHostToDevice));
                if (r >= 2) {
                    t_sel += t1 - t0;
                    t_sort += t2 - t1;
                    t_uni += t3 - t2;
                }
            }
            std::printf("n %7d bits %2d: host us per call  Flagged %6.1f  SortKeys %6.1f  Unique %6.1f\n", n, bits,
                        t_sel / reps, t_sort / reps, t_uni / reps);
        }
    }
    return 0;
}
