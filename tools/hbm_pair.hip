// Does a read-one / write-two stream (the GoL step's 4 B read + 8 B written
// per cell) run at the same rate in both directions between two buffers?
// Three 1 GiB buffers A, B, C (C at a byte offset `off` into a padded
// allocation); kernel X: B = f(A), C = g(A); kernel Y: A = f(B), C = g(B).
// usage: hbm_pair [plain|contig|blk|band2|band8|band32] [off_bytes ...]  (blk: k_rw_blk, bandN: k_rw_band<N>)  (contig: hipExtMallocWithFlags
// with hipDeviceMallocContiguous)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

__global__ void __launch_bounds__(256) k_rw(const uint4* __restrict__ in, uint4* __restrict__ o1, uint4* __restrict__ o2,
                                            size_t n4)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const uint4 v = in[i];
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 a = {v.x + 1, v.y + 1, v.z + 1, v.w + 1}, b = {v.x ^ 5, v.y ^ 5, v.z ^ 5, v.w ^ 5};
        __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(o1 + i));
        __builtin_nontemporal_store(b, reinterpret_cast<u32x4*>(o2 + i));
    }
}

// the same stream, each workgroup owning one contiguous span: the
// concurrently running workgroups touch addresses spread over the whole arrays
__global__ void __launch_bounds__(256) k_rw_blk(const uint4* __restrict__ in, uint4* __restrict__ o1,
                                                uint4* __restrict__ o2, size_t n4)
{
    const size_t per = (n4 + gridDim.x - 1) / gridDim.x, b0 = (size_t)blockIdx.x * per;
    const size_t b1 = b0 + per < n4 ? b0 + per : n4;
    for (size_t i = b0 + threadIdx.x; i < b1; i += 256) {
        const uint4 v = in[i];
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 a = {v.x + 1, v.y + 1, v.z + 1, v.w + 1}, b = {v.x ^ 5, v.y ^ 5, v.z ^ 5, v.w ^ 5};
        __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(o1 + i));
        __builtin_nontemporal_store(b, reinterpret_cast<u32x4*>(o2 + i));
    }
}

// grid-stride within BANDS equal bands, workgroup b in band b % BANDS: the
// running workgroups sit in BANDS separate places of the arrays
template <int BANDS>
__global__ void __launch_bounds__(256) k_rw_band(const uint4* __restrict__ in, uint4* __restrict__ o1,
                                                 uint4* __restrict__ o2, size_t n4)
{
    const size_t per = n4 / BANDS, b = blockIdx.x % BANDS, wb = blockIdx.x / BANDS, nb = gridDim.x / BANDS;
    for (size_t j = wb * 256 + threadIdx.x; j < per; j += nb * 256) {
        const size_t i = b * per + j;
        const uint4 v = in[i];
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 a = {v.x + 1, v.y + 1, v.z + 1, v.w + 1}, c = {v.x ^ 5, v.y ^ 5, v.z ^ 5, v.w ^ 5};
        __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(o1 + i));
        __builtin_nontemporal_store(c, reinterpret_cast<u32x4*>(o2 + i));
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char** argv)
{
    const size_t bytes = (size_t)1 << 30, n4 = bytes / 16;
    std::vector<size_t> offs;
    int a0 = 1;
    bool contig = false, blk = false;
    std::string mode = "plain";
    if (argc > 1 && !isdigit(argv[1][0])) {
        mode = argv[1];
        contig = mode == "contig";
        blk = mode == "blk";
        a0 = 2;
    }
    auto kern = blk ? k_rw_blk : mode == "band2" ? k_rw_band<2> : mode == "band8" ? k_rw_band<8>
              : mode == "band32" ? k_rw_band<32> : k_rw;
    auto alloc = [&](char** p, size_t b) {
        if (contig) CK(hipExtMallocWithFlags((void**)p, b, hipDeviceMallocContiguous));
        else CK(hipMalloc(p, b));
    };
    for (int i = a0; i < argc; i++) offs.push_back(strtoull(argv[i], nullptr, 0));
    if (offs.empty()) offs = {0};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (size_t off : offs) {
        char *A, *B, *C;
        alloc(&A, bytes + (2 << 20));
        alloc(&B, bytes + (2 << 20));
        alloc(&C, bytes + off + (2 << 20));
        CK(hipMemset(A, 1, bytes));
        CK(hipMemset(B, 2, bytes));
        char* Cp = C + off;
        const unsigned g = 256 * 16;
        float tx = 0, ty = 0, mx = 1e9, my = 1e9;
        const int reps = 20;
        for (int r = 0; r < reps + 2; r++) {
            float t;
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, (const uint4*)A, (uint4*)B, (uint4*)Cp, n4);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r >= 2) { tx += t; mx = t < mx ? t : mx; }
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, (const uint4*)B, (uint4*)A, (uint4*)Cp, n4);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r >= 2) { ty += t; my = t < my ? t : my; }
        }
        const double gb = 3.0 * bytes / 1e9;
        printf("%s C offset %8zu: A->B %.3f ms (%.0f GB/s, min %.3f)  B->A %.3f ms (%.0f GB/s, min %.3f)  A %p B %p C %p\n", mode.c_str(), off,
               tx / reps, gb / (tx / reps * 1e-3), mx, ty / reps, gb / (ty / reps * 1e-3), my, (void*)A, (void*)B,
               (void*)Cp);
        CK(hipFree(A));
        CK(hipFree(B));
        CK(hipFree(C));
    }
    return 0;
}
