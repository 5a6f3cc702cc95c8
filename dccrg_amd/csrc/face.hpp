// face.hpp -- the face graph and face neighbors as device functions over an
// existence predicate (the explicit grid's hash, or "level 0" for uniform
// grids), so one restatement serves both layouts.
#pragma once

#include "internal.hpp"

namespace dccrgx {

// Dccrg::get_existing_cell, dccrg.hpp:11414-11447: the smallest existing
// cell at indices idx within levels [lo, hi]
template <class Exists>
__host__ __device__ inline uint64_t existing_cell(const MapParams& mp, const uint64_t idx[3], int lo, int hi,
                                                  const Exists& exists)
{
    for (int l = hi; l >= lo; l--) {
        const uint64_t c = map_cell(mp, idx, l);  // 0 outside the grid
        if (c == 0) return 0;
        if (exists(c)) return c;
    }
    return 0;
}

// Dccrg::update_neighbors_(cell), dccrg.hpp:9463-9597: for -x, +x, -y, +y,
// -z, +z the existing cell adjacent to the face within one level, periodic
// wrap in index space; 0 (error_cell) where there is none or the cell is not
// an existing leaf
template <class Exists>
__host__ __device__ inline void face_graph(const MapParams& mp, const int32_t per[3], uint64_t cell, uint64_t out[6],
                                           const Exists& exists)
{
    for (int i = 0; i < 6; i++) out[i] = 0;
    uint64_t idx[3];
    int lvl;
    if (!map_indices(mp, cell, idx, &lvl) || !exists(cell)) return;
    const int M = mp.max_lvl;
    if (lvl < M && exists(map_cell(mp, idx, lvl + 1))) return;  // refined: not a leaf (get_child, :9694-9718)
    const uint64_t len = (uint64_t)1 << (M - lvl);
    const int lo = lvl == 0 ? 0 : lvl - 1, hi = lvl == M ? M : lvl + 1;
    for (int d = 0; d < 3; d++) {
        const uint64_t n_idx = mp.length[d] << M;  // indices along d
        for (int sg = 0; sg < 2; sg++) {
            uint64_t s[3] = {idx[0], idx[1], idx[2]};
            bool ok = true;
            if (sg == 0) {
                if (s[d] == 0) {
                    if (per[d]) s[d] = n_idx - 1;
                    else ok = false;
                } else {
                    s[d]--;
                }
            } else {
                const uint64_t max_index = n_idx - 1;
                if (max_index < len || s[d] > max_index - len) {
                    if (per[d]) s[d] = 0;
                    else ok = false;
                } else {
                    s[d] += len;
                }
            }
            out[2 * d + sg] = ok ? existing_cell(mp, s, lo, hi, exists) : 0;
        }
    }
}

// Dccrg::get_face_neighbors_of, dccrg.hpp:2828-2955: the face-graph neighbor
// of each direction and, when it is smaller, its three siblings sharing the
// face (reached through its own face graph).  Direction codes -1, +1, -2, +2,
// -3, +3.  At most 24 entries; returns the count.
template <class Exists>
__host__ __device__ inline int face_neighbors(const MapParams& mp, const int32_t per[3], uint64_t cell,
                                              uint64_t ids[24], int32_t dirs[24], const Exists& exists)
{
    uint64_t ng[6];
    face_graph(mp, per, cell, ng, exists);
    const int lvl = map_level(mp, cell);
    int n = 0;
    for (int i = 0; i < 6; i++) {
        const uint64_t nb = ng[i];
        if (nb == 0) continue;
        const int32_t dir = (i & 1) ? (i / 2 + 1) : -(i / 2 + 1);
        ids[n] = nb;
        dirs[n++] = dir;
        if (lvl >= map_level(mp, nb)) continue;
        // the two tangential positive directions (:2874-2946)
        const int a = i < 2 ? 3 : 1, b = i < 4 ? 5 : 3;
        uint64_t nn[6];
        face_graph(mp, per, nb, nn, exists);
        if (nn[a]) {
            ids[n] = nn[a];
            dirs[n++] = dir;
        }
        if (nn[b]) {
            ids[n] = nn[b];
            dirs[n++] = dir;
            uint64_t nnn[6];
            face_graph(mp, per, nn[b], nnn, exists);
            if (nnn[a]) {
                ids[n] = nnn[a];
                dirs[n++] = dir;
            }
        }
    }
    return n;
}

// batched get_face_neighbors_of: pass 1 (ids == nullptr) counts into
// row[i + 1], pass 2 fills at row[i]; err |= 1 for a cell that is not an
// existing leaf (the reference aborts, dccrg.hpp:2845-2849)
template <class Exists>
__global__ void __launch_bounds__(256) k_face_nbrs(MapParams mp, int32_t px, int32_t py, int32_t pz, Exists exists,
                                                   const uint64_t* __restrict__ cells, size_t n,
                                                   uint64_t* __restrict__ row, uint64_t* __restrict__ ids,
                                                   int32_t* __restrict__ dirs, int32_t* __restrict__ err)
{
    const int32_t per[3] = {px, py, pz};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t c = cells[i];
        uint64_t fid[24];
        int32_t fd[24];
        int k = 0;
        if (map_level(mp, c) < 0 || !exists(c)) atomicOr(err, 1);
        else k = face_neighbors(mp, per, c, fid, fd, exists);
        if (!ids) {
            row[i + 1] = (uint64_t)k;
            continue;
        }
        const uint64_t w = row[i];
        for (int j = 0; j < k; j++) {
            ids[w + j] = fid[j];
            if (dirs) dirs[w + j] = fd[j];
        }
    }
}

template <class Exists>
int face_neighbors_launch(const MapParams& mp, const uint8_t periodic[3], const Exists& exists,
                          const uint64_t* cells, size_t n, uint64_t* row, uint64_t* ids, int32_t* dirs,
                          size_t cap, hipStream_t st)
{
    uint64_t g = (n + 255) / 256;
    g = g == 0 ? 1 : (g > 4096 ? 4096 : g);
    int32_t* d_err = nullptr;
    DX_HIP(dx_malloc(&d_err, 4));
    DX_HIP(hipMemsetAsync(d_err, 0, 4, st));
    DX_HIP(hipMemsetAsync(row, 0, 8, st));
    if (n)
        hipLaunchKernelGGL(k_face_nbrs<Exists>, dim3((unsigned)g), dim3(256), 0, st, mp, (int32_t)periodic[0],
                           (int32_t)periodic[1], (int32_t)periodic[2], exists, cells, n, row, (uint64_t*)nullptr,
                           (int32_t*)nullptr, d_err);
    DX_HIP(hipGetLastError());
    std::vector<uint64_t> h(n + 1);
    int32_t err = 0;
    DX_HIP(hipMemcpyAsync(h.data(), row, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    DX_HIP(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
    DX_HIP(hipStreamSynchronize(st));
    if (err) dx_free(d_err);
    DX_CHECK(!err, DCCRGX_ENOTFOUND, "cell is not an existing leaf");
    h[0] = 0;
    for (size_t i = 0; i < n; i++) h[i + 1] += h[i];
    DX_HIP(hipMemcpyAsync(row, h.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
    int s = DCCRGX_OK;
    if (ids && cap < h[n])
        s = set_error(DCCRGX_ERANGE, "capacity %zu < %llu", cap, (unsigned long long)h[n]);
    else if (ids && n)
        hipLaunchKernelGGL(k_face_nbrs<Exists>, dim3((unsigned)g), dim3(256), 0, st, mp, (int32_t)periodic[0],
                           (int32_t)periodic[1], (int32_t)periodic[2], exists, cells, n, row, ids, dirs, d_err);
    DX_HIP(hipGetLastError());
    DX_HIP(hipStreamSynchronize(st));
    dx_free(d_err);
    return s;
}

}  // namespace dccrgx
