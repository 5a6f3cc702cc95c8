// sfc.hip -- space-filling-curve placement of the level-0 cells (SURVEY 8(f)
// row 4; the reference's USE_SFC branch of create_level_0_cells,
// dccrg.hpp:8147-8220).
//
// The reference walks the level-0 cells in the order of sfc++'s curve and
// gives each process the same number of consecutive cells as its block
// partition (cells_per_process, procs_with_fewer: :8098-8114), recording the
// owner of every cell in the replicated cell_process map.  sfc++ is not part
// of the reference tree, so its curve cannot be reproduced; here the curve is
// the 3-D Hilbert curve (hilbert3, internal.hpp) over the smallest
// power-of-two cube holding the grid, cells outside the grid skipped.
//
// No per-cell state is kept.  Process r owns the cells at curve positions
// [first_r, first_{r+1}); keys grow with the position, so the P - 1 keys of
// the cells at first_1 .. first_{P-1} (the cuts) decide every owner:
// owner(cell) = number of cuts <= key(cell) (sfc_owner, host and device).
// A cut is found without enumerating cells: the number of grid cells whose
// key is below K is a sum over the Hilbert octree (every key prefix is an
// aligned sub-cube, so the sub-cubes left of K's path contribute their
// overlap with the grid box), and the key at position s is the smallest K
// with count_below(K + 1) > s (binary search over the key range).  That is
// O(P * 3b * 8b * b) host arithmetic at grid creation, no device memory.
#include "grid.hpp"

namespace dccrgx {

namespace {

// Skilling's transpose-to-axes: the cell (X[0], X[1], X[2]) of Hilbert key
// `key` (inverse of hilbert3)
void hilbert3_axes(uint64_t key, int b, uint32_t X[3])
{
    X[0] = X[1] = X[2] = 0;
    for (int bit = b - 1; bit >= 0; bit--)
        for (int i = 0; i < 3; i++) X[i] = (X[i] << 1) | (uint32_t)((key >> (3 * bit + 2 - i)) & 1u);
    const uint32_t N = 2u << (b - 1);
    uint32_t t = X[2] >> 1;  // Gray decode
    for (int i = 2; i > 0; i--) X[i] ^= X[i - 1];
    X[0] ^= t;
    for (uint32_t Q = 2; Q != N; Q <<= 1) {  // undo excess work
        const uint32_t P = Q - 1;
        for (int i = 2; i >= 0; i--) {
            if (X[i] & Q) {
                X[0] ^= P;
            } else {
                t = (X[0] ^ X[i]) & P;
                X[0] ^= t;
                X[i] ^= t;
            }
        }
    }
}

// number of grid cells with a key below K (K <= 8^b)
uint64_t count_below(uint64_t K, int b, const uint64_t L[3])
{
    if (K >> (3 * b)) return L[0] * L[1] * L[2];
    uint64_t total = 0;
    for (int l = 0; l < b; l++) {
        const int shift = 3 * (b - 1 - l);
        const uint64_t digit = (K >> shift) & 7u, hi = (K >> shift) & ~7ull;
        const uint64_t side = 1ull << (b - 1 - l);
        for (uint64_t j = 0; j < digit; j++) {  // sub-cubes entirely below K at this level
            uint32_t X[3];
            hilbert3_axes((hi | j) << shift, b, X);
            uint64_t vol = 1;
            for (int a = 0; a < 3 && vol; a++) {
                const uint64_t o = (uint64_t)X[a] & ~(side - 1);
                vol *= o < L[a] ? std::min(o + side, L[a]) - o : 0;
            }
            total += vol;
        }
    }
    return total;
}

// key of the grid cell at curve position s (s < the number of cells)
uint64_t key_at(uint64_t s, int b, const uint64_t L[3])
{
    uint64_t lo = 0, hi = (1ull << (3 * b)) - 1;  // smallest K with count_below(K + 1) > s
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (count_below(mid + 1, b, L) > s)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

}  // namespace

int sfc_plan(const uint64_t length[3], int comm_size, SfcPlan& out)
{
    const uint64_t n = length[0] * length[1] * length[2];
    DX_CHECK(n > 0 && n < (1ull << 32), DCCRGX_EINVAL, "SFC placement of %llu level-0 cells",
             (unsigned long long)n);
    DX_CHECK(comm_size > 0, DCCRGX_EINVAL, "comm size %d", comm_size);
    const uint64_t side = std::max(length[0], std::max(length[1], length[2]));
    int b = 1;
    while ((1ull << b) < side) b++;
    DX_CHECK(b <= 21, DCCRGX_EINVAL, "grid side %llu too long for 64-bit Hilbert keys", (unsigned long long)side);
    SfcPlan p;
    p.bits = b;
    std::copy(length, length + 3, p.length);
    p.div_lx = make_divider(length[0]);
    p.div_lxly = make_divider(length[0] * length[1]);
    p.enabled = true;
    const Partition P = make_partition(n, comm_size);
    p.cut.resize(comm_size - 1);
    uint64_t prev_s = ~0ull, prev_key = 0;
    for (int r = 1; r < comm_size; r++) {
        const uint64_t s = part_first(P, r) - 1;  // process r's first curve position
        if (s >= n) {
            p.cut[r - 1] = ~0ull;  // no cells (never <= a key: keys are below 2^63)
            continue;
        }
        if (s != prev_s) {  // processes with no cells repeat the next one's cut
            prev_key = key_at(s, b, length);
            prev_s = s;
        }
        p.cut[r - 1] = prev_key;
    }
    out = std::move(p);
    return DCCRGX_OK;
}

}  // namespace dccrgx

using namespace dccrgx;

extern "C" {

int dccrgx_hilbert_keys_host(const uint64_t length[3], uint64_t* keys_out)
{
    DX_CHECK(length && keys_out, DCCRGX_EINVAL, "null argument");
    const uint64_t n = length[0] * length[1] * length[2];
    const uint64_t side = std::max(length[0], std::max(length[1], length[2]));
    int b = 1;
    while ((1ull << b) < side) b++;
    DX_CHECK(b <= 21, DCCRGX_EINVAL, "grid side too long");
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = i % length[0], y = (i / length[0]) % length[1], z = i / (length[0] * length[1]);
        keys_out[i] = hilbert3((uint32_t)x, (uint32_t)y, (uint32_t)z, b);
    }
    return DCCRGX_OK;
}

int dccrgx_sfc_cuts(const uint64_t length[3], int32_t comm_size, uint64_t* cuts_out)
{
    DX_CHECK(length && (cuts_out || comm_size == 1), DCCRGX_EINVAL, "null argument");
    SfcPlan p;
    DX_TRY(sfc_plan(length, comm_size, p));
    std::copy(p.cut.begin(), p.cut.end(), cuts_out);
    return DCCRGX_OK;
}

int dccrgx_sfc_owners(dccrgx_ctx* ctx, const uint64_t length[3], int32_t comm_size, int32_t* owner_host)
{
    (void)ctx;  // host arithmetic: kept in the signature for callers of the table form
    DX_CHECK(length && owner_host, DCCRGX_EINVAL, "null argument");
    SfcPlan p;
    DX_TRY(sfc_plan(length, comm_size, p));
    const SfcCuts s = p.view();
    const uint64_t n = length[0] * length[1] * length[2];
    for (uint64_t i = 0; i < n; i++) owner_host[i] = sfc_owner(s, i + 1);
    return DCCRGX_OK;
}

}  // extern "C"
