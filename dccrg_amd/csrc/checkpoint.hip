// checkpoint.hip -- dccrg's grid data files: save_grid_data, and
// start_loading_grid_data / continue_loading_grid_data /
// finish_loading_grid_data (dccrg.hpp:1109-2427), byte-compatible with the
// reference's file layout (see include/dccrgx.h and oracle/dccrg_checkpoint.py).
//
// The reference builds one MPI struct datatype over every local cell's
// get_mpi_datatype() and writes it through MPI-IO.  Here cell data lives in
// device SoA fields, so a cell's record (its fields' bytes in the order
// given, no padding -- the packed form of the struct datatype, :1385-1420)
// is assembled by a device kernel into a staging buffer, copied to the host
// in large chunks and written with one pwrite per chunk: a rank's records
// are contiguous in the file (rank by rank, cells in the rank's order,
// :1500-1520).  Loading reads each local cell's record at the offset the
// file's cell list gives (any order, any writer rank count) and a device
// kernel scatters the records into the fields.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstring>

#include "grid.hpp"

namespace dccrgx {

struct LoadState {
    std::string path;
    std::vector<uint64_t> disp;  // file offset of the next unread byte of each local cell (local order)
    bool affine = false;         // disp[i] = disp[0] + i * stride
    uint64_t stride = 0;
};

namespace {

constexpr uint64_t ENDIANNESS = 0x1234567890abcdefull;
constexpr int MAXF = 16;
constexpr uint64_t CHUNK_BYTES = 256ull << 20;

struct FDesc {
    char* ptr[MAXF];
    uint32_t elem[MAXF];
    uint32_t off[MAXF];  // byte offset inside the record
    int32_t nf;
    uint32_t rec;        // record bytes
};

unsigned blocks_for(uint64_t n)
{
    uint64_t g = (n + 255) / 256;
    if (g > 256 * 64) g = 256 * 64;
    if (g == 0) g = 1;
    return (unsigned)g;
}

// records of cells [i0, i0 + n) (slot s0 + i) <-> staging buffer; one thread
// per 4-byte word of the staging buffer when every size is a multiple of 4
// (coalesced on the staging side), else per byte
template <bool PACK, class W>
__global__ void __launch_bounds__(256) k_records(FDesc d, uint64_t s0, uint64_t i0, uint64_t n, char* __restrict__ buf)
{
    const uint64_t words = d.rec / sizeof(W);
    const uint64_t tot = n * words;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += stride) {
        const uint64_t c = t / words, w = (t - c * words) * sizeof(W);
        int k = 0;
        while (k + 1 < d.nf && d.off[k + 1] <= w) k++;
        const uint64_t fb = w - d.off[k];
        W* f = (W*)(d.ptr[k] + (s0 + i0 + c) * d.elem[k] + fb);
        W* b = (W*)(buf + t * sizeof(W));
        if (PACK) *b = *f;
        else *f = *b;
    }
}

int fdesc(const dccrgx_grid* g, const int32_t* f, size_t nf, FDesc* d, bool* variable)
{
    DX_CHECK(f || !nf, DCCRGX_EINVAL, "null field list");
    DX_CHECK(nf <= (size_t)MAXF, DCCRGX_EINVAL, "at most %d fields per record", MAXF);
    *variable = false;
    std::memset(d, 0, sizeof(*d));
    d->nf = (int32_t)nf;
    uint32_t off = 0;
    for (size_t i = 0; i < nf; i++) {
        DX_CHECK(f[i] >= 0 && (size_t)f[i] < g->fields.size(), DCCRGX_EINVAL, "bad field %d", f[i]);
        const Field& F = g->fields[f[i]];
        *variable |= F.variable;
        d->ptr[i] = (char*)F.ptr;
        d->elem[i] = F.elem;
        d->off[i] = off;
        off += F.elem;
    }
    d->rec = off;
    return DCCRGX_OK;
}

// first storage slot of the local cells (local position i <-> slot s0 + i)
uint64_t local_s0(const dccrgx_grid* g)
{
    if (!g->uniform) return 0;
    return g->g.lo + (uint64_t)(-g->g.cbase * (int64_t)g->g.S);
}

uint64_t local_id(const dccrgx_grid* g, uint64_t i) { return g->uniform ? g->first_local + i : g->ex->local()[i]; }

// record bytes of local cell i
uint64_t record_bytes(const dccrgx_grid* g, const int32_t* f, size_t nf, uint64_t s0, uint64_t i)
{
    uint64_t b = 0;
    for (size_t k = 0; k < nf; k++) {
        const Field& F = g->fields[f[k]];
        b += F.variable ? (uint64_t)F.count[s0 + i] * F.elem : F.elem;
    }
    return b;
}

int pwrite_all(int fd, const void* p, uint64_t n, uint64_t at)
{
    const char* c = (const char*)p;
    while (n) {
        const ssize_t w = pwrite(fd, c, std::min<uint64_t>(n, 1ull << 30), (off_t)at);
        DX_CHECK(w > 0, DCCRGX_EINVAL, "write failed at byte %llu", (unsigned long long)at);
        c += w;
        n -= (uint64_t)w;
        at += (uint64_t)w;
    }
    return DCCRGX_OK;
}

int pread_all(int fd, void* p, uint64_t n, uint64_t at)
{
    char* c = (char*)p;
    while (n) {
        const ssize_t r = pread(fd, c, std::min<uint64_t>(n, 1ull << 30), (off_t)at);
        DX_CHECK(r > 0, DCCRGX_EINVAL, "file ends before byte %llu", (unsigned long long)(at + n));
        c += r;
        n -= (uint64_t)r;
        at += (uint64_t)r;
    }
    return DCCRGX_OK;
}

struct Fd {
    int fd = -1;
    ~Fd()
    {
        if (fd >= 0) close(fd);
    }
};

// data_size() of the geometry whose id is at `p` (dccrg_no_geometry.hpp:547,
// dccrg_cartesian_geometry.hpp:810, dccrg_stretched_cartesian_geometry.hpp:808)
int geometry_bytes(int fd, uint64_t at, uint64_t* out)
{
    int32_t id = -1;
    DX_TRY(pread_all(fd, &id, 4, at));
    if (id == 0) *out = 4;
    else if (id == 1) *out = 4 + 48;
    else if (id == 2) {
        uint64_t n[3];
        DX_TRY(pread_all(fd, n, 24, at + 4));
        *out = 4 + 24 + 8 * (n[0] + n[1] + n[2]);
    } else {
        return set_error(DCCRGX_EINVAL, "unknown geometry id %d", id);
    }
    return DCCRGX_OK;
}

// staging for one direction of a chunk: device buffer + pinned host buffer
struct Staging {
    char* d = nullptr;
    char* h = nullptr;
    uint64_t cap = 0;
    ~Staging()
    {
        dx_free(d);
        hipHostFree(h);
    }
    int ensure(uint64_t n)
    {
        if (n <= cap) return DCCRGX_OK;
        dx_free(d);
        hipHostFree(h);
        d = h = nullptr;
        cap = 0;
        DX_HIP(dx_malloc(&d, n));
        DX_HIP(hipHostMalloc(&h, n));
        cap = n;
        return DCCRGX_OK;
    }
};

template <bool PACK>
int launch_records(const FDesc& d, uint64_t s0, uint64_t i0, uint64_t n, char* buf, hipStream_t st)
{
    if (!n || !d.rec) return DCCRGX_OK;
    bool w4 = d.rec % 4 == 0;
    for (int k = 0; k < d.nf; k++) w4 &= d.elem[k] % 4 == 0;
    if (w4)
        hipLaunchKernelGGL((k_records<PACK, uint32_t>), dim3(blocks_for(n * d.rec / 4)), dim3(256), 0, st, d, s0, i0,
                           n, buf);
    else
        hipLaunchKernelGGL((k_records<PACK, uint8_t>), dim3(blocks_for(n * d.rec)), dim3(256), 0, st, d, s0, i0, n,
                           buf);
    DX_HIP(hipGetLastError());
    return DCCRGX_OK;
}

// variable-size records: host-built byte segments (field <-> staging)
struct VSeg {
    uint64_t a, b, len;  // device byte offsets: field pool, staging
};

__global__ void __launch_bounds__(256) k_vsegs(const VSeg* __restrict__ s, uint64_t n, char* __restrict__ pool,
                                               char* __restrict__ buf, int pack)
{
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x % 64;
    const uint64_t waves = (uint64_t)gridDim.x * blockDim.x / 64;
    for (uint64_t k = wave; k < n; k += waves) {
        const VSeg v = s[k];
        for (uint64_t i = lane; i < v.len; i += 64) {
            if (pack) buf[v.b + i] = pool[v.a + i];
            else pool[v.a + i] = buf[v.b + i];
        }
    }
}

// records of cells [i0, i1) with at least one variable field: per (cell, field) segments
int var_records(const dccrgx_grid* g, const int32_t* f, size_t nf, uint64_t s0, uint64_t i0, uint64_t i1,
                char* dbuf, bool pack, hipStream_t st)
{
    for (size_t k = 0; k < nf; k++) {
        const Field& F = g->fields[f[k]];
        std::vector<VSeg> segs;
        uint64_t at = 0;
        for (uint64_t i = i0; i < i1; i++) {
            uint64_t before = 0;
            for (size_t j = 0; j < k; j++) {
                const Field& G = g->fields[f[j]];
                before += G.variable ? (uint64_t)G.count[s0 + i] * G.elem : G.elem;
            }
            const uint64_t len = F.variable ? (uint64_t)F.count[s0 + i] * F.elem : F.elem;
            const uint64_t src = F.variable ? F.off[s0 + i] : (s0 + i) * F.elem;
            if (len) segs.push_back({src, at + before, len});
            at += record_bytes(g, f, nf, s0, i);
        }
        if (segs.empty()) continue;
        VSeg* d = nullptr;
        DX_HIP(dx_malloc(&d, segs.size() * sizeof(VSeg)));
        DX_HIP(hipMemcpyAsync(d, segs.data(), segs.size() * sizeof(VSeg), hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_vsegs, dim3((unsigned)std::min<uint64_t>((segs.size() + 3) / 4, 4096)), dim3(256), 0, st,
                           d, (uint64_t)segs.size(), (char*)F.ptr, dbuf, pack ? 1 : 0);
        DX_HIP(hipGetLastError());
        DX_HIP(hipStreamSynchronize(st));
        dx_free(d);
    }
    return DCCRGX_OK;
}

}  // namespace

void load_state_free(dccrgx_grid* grid)
{
    delete grid->load;
    grid->load = nullptr;
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

uint64_t dccrgx_file_preamble_bytes(size_t geometry_bytes)
{
    // endianness 8, mapping 24 + 4, neighborhood length 4, topology 3, geometry, total cells 8
    return 8 + 28 + 4 + 3 + (uint64_t)geometry_bytes + 8;
}

int dccrgx_save_sizes(const dccrgx_grid* grid, const int32_t* fields, size_t nf, uint64_t* n_cells,
                      uint64_t* n_bytes)
{
    DX_CHECK(grid && n_cells && n_bytes, DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_TRY(explicit_host_leaves(grid));
    FDesc d;
    bool var = false;
    DX_TRY(fdesc(grid, fields, nf, &d, &var));
    *n_cells = grid->n_local;
    if (!var) {
        *n_bytes = grid->n_local * d.rec;
        return DCCRGX_OK;
    }
    const uint64_t s0 = local_s0(grid);
    uint64_t b = 0;
    for (uint64_t i = 0; i < grid->n_local; i++) b += record_bytes(grid, fields, nf, s0, i);
    *n_bytes = b;
    return DCCRGX_OK;
}

}  // extern "C"

namespace dccrgx {
namespace {

// save_grid_data's header, preamble (rank 0) and this rank's cell list;
// rec(i) = record bytes of local cell i.  Returns the file offset of the
// rank's first record.
template <class Rec>
int write_head_and_list(const dccrgx_grid* grid, int fd, uint64_t offset, const void* header, size_t header_bytes,
                        const void* geometry, size_t geometry_bytes, uint64_t total_cells, uint64_t cells_before,
                        uint64_t bytes_before, Rec rec, uint64_t* data_start_out)
{
    DX_CHECK(cells_before + grid->n_local <= total_cells, DCCRGX_EINVAL, "cell counts inconsistent");
    const uint64_t pre = offset + header_bytes + dccrgx_file_preamble_bytes(geometry_bytes);
    if (grid->ctx->rank == 0) {
        // rank 0: header, endianness check, mapping, neighborhood length,
        // topology, geometry, total number of cells (:1162-1310)
        std::vector<char> b(header_bytes + dccrgx_file_preamble_bytes(geometry_bytes));
        char* p = b.data();
        if (header_bytes) std::memcpy(p, header, header_bytes);
        p += header_bytes;
        std::memcpy(p, &ENDIANNESS, 8);
        p += 8;
        std::memcpy(p, grid->params.length, 24);
        p += 24;
        const int32_t mrl = grid->map.max_lvl;
        std::memcpy(p, &mrl, 4);
        p += 4;
        const uint32_t hl = grid->params.neighborhood_length;
        std::memcpy(p, &hl, 4);
        p += 4;
        for (int k = 0; k < 3; k++) *p++ = grid->params.periodic[k] ? 1 : 0;
        std::memcpy(p, geometry, geometry_bytes);
        p += geometry_bytes;
        std::memcpy(p, &total_cells, 8);
        DX_TRY(pwrite_all(fd, b.data(), b.size(), offset));
    }
    const uint64_t n = grid->n_local;
    const uint64_t list_start = pre + 16 * cells_before;
    const uint64_t data_start = pre + 16 * total_cells + bytes_before;
    // cell list: (id, absolute offset of its data) (:1540-1575)
    const uint64_t chunk = 1ull << 20;
    std::vector<uint64_t> pairs;
    uint64_t at = data_start;
    for (uint64_t i0 = 0; i0 < n; i0 += chunk) {
        const uint64_t i1 = std::min(n, i0 + chunk);
        pairs.resize(2 * (i1 - i0));
        for (uint64_t i = i0; i < i1; i++) {
            pairs[2 * (i - i0)] = local_id(grid, i);
            pairs[2 * (i - i0) + 1] = at;
            at += rec(i);
        }
        DX_TRY(pwrite_all(fd, pairs.data(), pairs.size() * 8, list_start + 16 * i0));
    }
    *data_start_out = data_start;
    return DCCRGX_OK;
}

}  // namespace
}  // namespace dccrgx

extern "C" {

int dccrgx_save_grid_data(const dccrgx_grid* grid, const char* path, uint64_t offset, const void* header,
                          size_t header_bytes, const void* geometry, size_t geometry_bytes, uint64_t total_cells,
                          uint64_t cells_before, uint64_t bytes_before, const int32_t* fields, size_t nf)
{
    DX_CHECK(grid && path && (header || !header_bytes) && geometry && geometry_bytes >= 4, DCCRGX_EINVAL,
             "null argument");
    DX_NO_HYBRID(grid);
    DX_TRY(explicit_host_leaves(grid));
    FDesc d;
    bool var = false;
    DX_TRY(fdesc(grid, fields, nf, &d, &var));
    Fd fd;
    // MPI_MODE_CREATE | MPI_MODE_WRONLY: no truncation (:1146-1152)
    fd.fd = open(path, O_WRONLY | O_CREAT, 0644);
    DX_CHECK(fd.fd >= 0, DCCRGX_EINVAL, "couldn't open file %s", path);
    const uint64_t n = grid->n_local;
    const uint64_t s0 = local_s0(grid);
    uint64_t data_start = 0;
    DX_TRY(write_head_and_list(
        grid, fd.fd, offset, header, header_bytes, geometry, geometry_bytes, total_cells, cells_before, bytes_before,
        [&](uint64_t i) { return var ? record_bytes(grid, fields, nf, s0, i) : (uint64_t)d.rec; }, &data_start));
    // cell data: records packed on the device, chunk by chunk
    hipStream_t st = grid->ctx->compute;
    Staging S;
    uint64_t at = data_start;
    if (!var) {
        if (!d.rec) return DCCRGX_OK;
        const uint64_t per = std::max<uint64_t>(1, CHUNK_BYTES / d.rec);
        DX_TRY(S.ensure(std::min(n, per) * d.rec));
        for (uint64_t i0 = 0; i0 < n; i0 += per) {
            const uint64_t m = std::min(n - i0, per);
            if (nf == 1)  // one field: the records are the field's slot run
                DX_HIP(hipMemcpyAsync(S.h, d.ptr[0] + (s0 + i0) * d.rec, m * d.rec, hipMemcpyDeviceToHost, st));
            else {
                DX_TRY(launch_records<true>(d, s0, i0, m, S.d, st));
                DX_HIP(hipMemcpyAsync(S.h, S.d, m * d.rec, hipMemcpyDeviceToHost, st));
            }
            DX_HIP(hipStreamSynchronize(st));
            DX_TRY(pwrite_all(fd.fd, S.h, m * d.rec, at));
            at += m * d.rec;
        }
        return DCCRGX_OK;
    }
    for (uint64_t i0 = 0; i0 < n;) {
        uint64_t i1 = i0, bytes = 0;
        while (i1 < n && (i1 == i0 || bytes + record_bytes(grid, fields, nf, s0, i1) <= CHUNK_BYTES))
            bytes += record_bytes(grid, fields, nf, s0, i1++);
        DX_TRY(S.ensure(std::max<uint64_t>(bytes, 1)));
        DX_TRY(var_records(grid, fields, nf, s0, i0, i1, S.d, true, st));
        DX_HIP(hipMemcpyAsync(S.h, S.d, bytes, hipMemcpyDeviceToHost, st));
        DX_HIP(hipStreamSynchronize(st));
        DX_TRY(pwrite_all(fd.fd, S.h, bytes, at));
        at += bytes;
        i0 = i1;
    }
    return DCCRGX_OK;
}

int dccrgx_file_read_info(const char* path, uint64_t offset, void* header, size_t header_bytes,
                          dccrgx_file_info* info, void* geometry, size_t geometry_cap)
{
    DX_CHECK(path && info && (header || !header_bytes), DCCRGX_EINVAL, "null argument");
    Fd fd;
    fd.fd = open(path, O_RDONLY);
    DX_CHECK(fd.fd >= 0, DCCRGX_ENOTFOUND, "couldn't open file %s", path);
    std::memset(info, 0, sizeof(*info));
    uint64_t at = offset;
    if (header_bytes) DX_TRY(pread_all(fd.fd, header, header_bytes, at));
    at += header_bytes;
    uint64_t e = 0;
    DX_TRY(pread_all(fd.fd, &e, 8, at));
    // :1925-1935
    DX_CHECK(e == ENDIANNESS, DCCRGX_EINVAL, "file %s has wrong endianness (0x%llx)", path, (unsigned long long)e);
    at += 8;
    DX_TRY(pread_all(fd.fd, info->params.length, 24, at));
    at += 24;
    DX_TRY(pread_all(fd.fd, &info->params.max_ref_lvl, 4, at));
    at += 4;
    DX_TRY(pread_all(fd.fd, &info->params.neighborhood_length, 4, at));
    at += 4;
    DX_TRY(pread_all(fd.fd, info->params.periodic, 3, at));
    for (int k = 0; k < 3; k++) info->params.periodic[k] = info->params.periodic[k] ? 1 : 0;
    at += 3;
    uint64_t gb = 0;
    DX_TRY(geometry_bytes(fd.fd, at, &gb));
    info->geometry_bytes = gb;
    if (geometry) {
        DX_CHECK(geometry_cap >= gb, DCCRGX_ERANGE, "geometry needs %llu bytes", (unsigned long long)gb);
        DX_TRY(pread_all(fd.fd, geometry, gb, at));
    }
    at += gb;
    DX_TRY(pread_all(fd.fd, &info->total_cells, 8, at));
    at += 8;
    info->list_offset = at;
    DX_CHECK(info->total_cells > 0, DCCRGX_EINVAL, "file %s lists no cells", path);
    return DCCRGX_OK;
}

int dccrgx_grid_load(dccrgx_ctx* ctx, const char* path, const dccrgx_file_info* info, dccrgx_grid** out)
{
    DX_CHECK(ctx && path && info && out, DCCRGX_EINVAL, "null argument");
    DX_CHECK(info->params.partition == DCCRGX_PARTITION_BLOCK || info->params.partition == DCCRGX_PARTITION_SFC,
             DCCRGX_EINVAL, "unknown placement %d", (int)info->params.partition);
    *out = nullptr;
    Fd fd;
    fd.fd = open(path, O_RDONLY);
    DX_CHECK(fd.fd >= 0, DCCRGX_ENOTFOUND, "couldn't open file %s", path);
    dccrgx_mapping m{};
    std::memcpy(m.length, info->params.length, 24);
    m.max_ref_lvl = info->params.max_ref_lvl;
    MapParams mp;
    DX_TRY(make_map_params(&m, &mp));
    const Partition part = make_partition(mp.nlevel0, ctx->comm_size);
    // the file records no placement: the loading grid's own (block, or the
    // SFC table of info->params) decides which rank reads which cells, as the
    // reference's load places cells by the new grid's partition
    SfcPlan sfc;
    if (info->params.partition == DCCRGX_PARTITION_SFC) DX_TRY(sfc_plan(info->params.length, ctx->comm_size, sfc));
    const SfcCuts sfc_cuts = sfc.view();
    // every cell in the list (:2033-2057); this rank loads the cells whose
    // level-0 ancestor is local (cell_overlaps_local, :2059-2071).  Pass 1
    // streams the list: are all cells level 0, and are this rank's cells
    // listed in ascending consecutive order with evenly spaced records (what
    // a save of a uniform grid produces)?  Only otherwise are ids stored.
    const uint64_t total = info->total_cells;
    const uint64_t chunk = 1ull << 20;
    std::vector<uint64_t> pairs;
    auto for_list = [&](auto&& visit) -> int {
        for (uint64_t i0 = 0; i0 < total; i0 += chunk) {
            const uint64_t i1 = std::min(total, i0 + chunk);
            pairs.resize(2 * (i1 - i0));
            DX_TRY(pread_all(fd.fd, pairs.data(), pairs.size() * 8, info->list_offset + 16 * i0));
            for (uint64_t i = 0; i < i1 - i0; i++) DX_TRY(visit(i0 + i, pairs[2 * i], pairs[2 * i + 1]));
        }
        return DCCRGX_OK;
    };
    auto owner_of = [&](uint64_t c, int* lvl) {
        uint64_t idx[3];
        if (c == 0 || !map_indices(mp, c, idx, lvl)) return -1;
        const uint64_t l0 = *lvl == 0 ? c : map_cell(mp, idx, 0);
        return sfc.on() ? sfc_owner(sfc_cuts, l0) : part_owner(part, l0);
    };
    bool all_level0 = true, simple = true;
    uint64_t n_mine = 0, first = 0, d0 = 0, stride = 0;
    DX_TRY(for_list([&](uint64_t k, uint64_t c, uint64_t disp) -> int {
        int l = -1;
        const int o = owner_of(c, &l);
        DX_CHECK(o >= 0, DCCRGX_EINVAL, "invalid cell %llu in the cell list at index %llu", (unsigned long long)c,
                 (unsigned long long)k);
        all_level0 &= l == 0;
        if (o != ctx->rank) return DCCRGX_OK;
        if (n_mine == 0) {
            first = c;
            d0 = disp;
        } else if (n_mine == 1) {
            stride = disp - d0;
            simple &= c == first + 1 && disp > d0;
        } else {
            simple &= c == first + n_mine && disp == d0 + n_mine * stride;
        }
        n_mine++;
        return DCCRGX_OK;
    }));
    // SFC grids always use the explicit layout (their local cells are not a slab)
    const bool uniform = all_level0 && total == mp.nlevel0 && !sfc.on();
    std::vector<uint64_t> leaves;
    if (!uniform) {
        leaves.reserve(total);
        DX_TRY(for_list([&](uint64_t, uint64_t c, uint64_t) -> int {
            leaves.push_back(c);
            return DCCRGX_OK;
        }));
    }
    dccrgx_grid* g = nullptr;
    DX_TRY(dccrgx_grid_create(ctx, &info->params, uniform ? nullptr : leaves.data(), uniform ? 0 : leaves.size(), &g));
    auto fail = [&](int code) {
        dccrgx_grid_destroy(g);
        return code;
    };
    if (n_mine != g->n_local)
        return fail(set_error(DCCRGX_EINVAL, "file lists %llu cells of this rank, the grid has %llu",
                              (unsigned long long)n_mine, (unsigned long long)g->n_local));
    auto* L = new LoadState();
    g->load = L;
    L->path = path;
    if (simple && n_mine && first == local_id(g, 0)) {
        L->affine = true;
        L->stride = stride;
        L->disp.assign(1, d0);
        *out = g;
        return DCCRGX_OK;
    }
    L->disp.assign(g->n_local, ~0ull);
    const int s = for_list([&](uint64_t, uint64_t c, uint64_t disp) -> int {
        int l = -1;
        if (owner_of(c, &l) != ctx->rank) return DCCRGX_OK;
        int64_t i;
        if (g->uniform) i = (int64_t)(c - g->first_local);
        else {
            const std::vector<uint64_t>& loc = g->ex->local();
            auto it = std::lower_bound(loc.begin(), loc.end(), c);
            i = (it != loc.end() && *it == c) ? (int64_t)(it - loc.begin()) : -1;
        }
        DX_CHECK(i >= 0 && (uint64_t)i < g->n_local && L->disp[i] == ~0ull, DCCRGX_EINVAL,
                 "cell %llu is listed twice or is not a local leaf", (unsigned long long)c);
        L->disp[i] = disp;
        return DCCRGX_OK;
    });
    if (s != DCCRGX_OK) return fail(s);
    *out = g;
    return DCCRGX_OK;
}

int dccrgx_load_cell_data(dccrgx_grid* grid, const int32_t* fields, size_t nf)
{
    DX_NOT_PENDING(grid);
    DX_NO_HYBRID(grid);
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    DX_CHECK(grid->load, DCCRGX_ESTATE, "the grid was not loaded from a file (or loading finished)");
    FDesc d;
    bool var = false;
    DX_TRY(fdesc(grid, fields, nf, &d, &var));
    LoadState& L = *grid->load;
    Fd fd;
    fd.fd = open(L.path.c_str(), O_RDONLY);
    DX_CHECK(fd.fd >= 0, DCCRGX_ENOTFOUND, "couldn't open file %s", L.path.c_str());
    const uint64_t n = grid->n_local, s0 = local_s0(grid);
    hipStream_t st = grid->ctx->compute;
    Staging S;
    if (!var && L.affine && (n <= 1 || L.stride == d.rec)) {
        // the rank's records are contiguous in the file, in local order
        if (d.rec) {
            const uint64_t per = std::max<uint64_t>(1, CHUNK_BYTES / d.rec);
            DX_TRY(S.ensure(std::min(n, per) * d.rec));
            for (uint64_t i0 = 0; i0 < n; i0 += per) {
                const uint64_t m = std::min(n - i0, per);
                DX_TRY(pread_all(fd.fd, S.h, m * d.rec, L.disp[0] + i0 * d.rec));
                if (nf == 1)
                    DX_HIP(hipMemcpyAsync(d.ptr[0] + (s0 + i0) * d.rec, S.h, m * d.rec, hipMemcpyHostToDevice, st));
                else {
                    DX_HIP(hipMemcpyAsync(S.d, S.h, m * d.rec, hipMemcpyHostToDevice, st));
                    DX_TRY(launch_records<false>(d, s0, i0, m, S.d, st));
                }
                DX_HIP(hipStreamSynchronize(st));
            }
        }
        L.disp[0] += d.rec;  // continue_loading_grid_data moves every offset (:2235-2248)
        return DCCRGX_OK;
    }
    // general: records gathered into local order from wherever the file has them
    for (uint64_t i0 = 0; i0 < n;) {
        uint64_t i1 = i0, bytes = 0;
        while (i1 < n && (i1 == i0 || bytes + record_bytes(grid, fields, nf, s0, i1) <= CHUNK_BYTES))
            bytes += record_bytes(grid, fields, nf, s0, i1++);
        DX_TRY(S.ensure(std::max<uint64_t>(bytes, 1)));
        // (file offset, staging offset, length) of each cell, merged where contiguous in both
        std::vector<std::array<uint64_t, 3>> runs;
        uint64_t at = 0;
        std::vector<std::array<uint64_t, 3>> cells;
        for (uint64_t i = i0; i < i1; i++) {
            const uint64_t rb = record_bytes(grid, fields, nf, s0, i);
            const uint64_t src = L.affine ? L.disp[0] + i * L.stride : L.disp[i];
            if (rb) cells.push_back({src, at, rb});
            at += rb;
        }
        std::sort(cells.begin(), cells.end());
        for (auto& c : cells) {
            if (!runs.empty() && runs.back()[0] + runs.back()[2] == c[0] && runs.back()[1] + runs.back()[2] == c[1])
                runs.back()[2] += c[2];
            else
                runs.push_back(c);
        }
        for (auto& r : runs) DX_TRY(pread_all(fd.fd, S.h + r[1], r[2], r[0]));
        DX_HIP(hipMemcpyAsync(S.d, S.h, bytes, hipMemcpyHostToDevice, st));
        if (var) DX_TRY(var_records(grid, fields, nf, s0, i0, i1, S.d, false, st));
        else DX_TRY(launch_records<false>(d, s0, i0, i1 - i0, S.d, st));
        DX_HIP(hipStreamSynchronize(st));
        i0 = i1;
    }
    if (L.affine && !var) {
        L.disp[0] += d.rec;
    } else {
        if (L.affine) {  // per-cell offsets from here on
            const uint64_t d0 = L.disp[0];
            L.disp.resize(n);
            for (uint64_t i = 0; i < n; i++) L.disp[i] = d0 + i * L.stride;
            L.affine = false;
        }
        for (uint64_t i = 0; i < n; i++) L.disp[i] += record_bytes(grid, fields, nf, s0, i);
    }
    return DCCRGX_OK;
}

int dccrgx_finish_loading_grid_data(dccrgx_grid* grid)
{
    DX_CHECK(grid, DCCRGX_EINVAL, "null grid");
    DX_NO_HYBRID(grid);
    load_state_free(grid);
    return DCCRGX_OK;
}

int dccrgx_save_grid_data_host(const dccrgx_grid* grid, const char* path, uint64_t offset, const void* header,
                               size_t header_bytes, const void* geometry, size_t geometry_bytes, uint64_t total_cells,
                               uint64_t cells_before, uint64_t bytes_before, const uint64_t* record_bytes,
                               const void* records, size_t bytes)
{
    DX_CHECK(grid && path && (header || !header_bytes) && geometry && geometry_bytes >= 4 &&
                 (record_bytes || !grid->n_local) && (records || !bytes),
             DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_TRY(explicit_host_leaves(grid));
    uint64_t tot = 0;
    for (uint64_t i = 0; i < grid->n_local; i++) tot += record_bytes[i];
    DX_CHECK(tot == bytes, DCCRGX_EINVAL, "records hold %zu bytes, their sizes add up to %llu", bytes,
             (unsigned long long)tot);
    Fd fd;
    fd.fd = open(path, O_WRONLY | O_CREAT, 0644);
    DX_CHECK(fd.fd >= 0, DCCRGX_EINVAL, "couldn't open file %s", path);
    uint64_t data_start = 0;
    DX_TRY(write_head_and_list(grid, fd.fd, offset, header, header_bytes, geometry, geometry_bytes, total_cells,
                               cells_before, bytes_before, [&](uint64_t i) { return record_bytes[i]; }, &data_start));
    if (bytes) DX_TRY(pwrite_all(fd.fd, records, bytes, data_start));
    return DCCRGX_OK;
}

int dccrgx_load_cell_records_host(dccrgx_grid* grid, const uint64_t* record_bytes, void* out, size_t bytes)
{
    DX_CHECK(grid && (record_bytes || !grid->n_local) && (out || !bytes), DCCRGX_EINVAL, "null argument");
    DX_NO_HYBRID(grid);
    DX_CHECK(grid->load, DCCRGX_ESTATE, "the grid was not loaded from a file (or loading finished)");
    LoadState& L = *grid->load;
    const uint64_t n = grid->n_local;
    uint64_t tot = 0;
    for (uint64_t i = 0; i < n; i++) tot += record_bytes[i];
    DX_CHECK(tot == bytes, DCCRGX_EINVAL, "buffer holds %zu bytes, the records %llu", bytes, (unsigned long long)tot);
    Fd fd;
    fd.fd = open(L.path.c_str(), O_RDONLY);
    DX_CHECK(fd.fd >= 0, DCCRGX_ENOTFOUND, "couldn't open file %s", L.path.c_str());
    if (L.affine) {
        const uint64_t d0 = L.disp[0];
        L.disp.resize(n);
        for (uint64_t i = 0; i < n; i++) L.disp[i] = d0 + i * L.stride;
        L.affine = false;
    }
    std::vector<std::array<uint64_t, 3>> cells;  // (file offset, buffer offset, length), merged where contiguous
    uint64_t at = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (record_bytes[i]) cells.push_back({L.disp[i], at, record_bytes[i]});
        at += record_bytes[i];
        L.disp[i] += record_bytes[i];
    }
    std::sort(cells.begin(), cells.end());
    std::vector<std::array<uint64_t, 3>> runs;
    for (auto& c : cells) {
        if (!runs.empty() && runs.back()[0] + runs.back()[2] == c[0] && runs.back()[1] + runs.back()[2] == c[1])
            runs.back()[2] += c[2];
        else
            runs.push_back(c);
    }
    for (auto& r : runs) DX_TRY(pread_all(fd.fd, (char*)out + r[1], r[2], r[0]));
    return DCCRGX_OK;
}

}  // extern "C"
