/*
 * dccrg_oracle.c -- TEST INFRASTRUCTURE ONLY (see dccrg_oracle.h).
 *
 * Plain C restatement of the reference algorithms.  Deliberately written in
 * the reference's own style (loops, face-graph walk, per-call hashing) so that
 * it can serve as an independent checker of the MI355X-native product, which
 * computes the same results with entirely different (closed-form, batched)
 * algorithms.  Never used by the product path.
 */
#include "dccrg_oracle.h"

#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ========================================================================
 * Mapping -- dccrg_mapping.hpp
 * ====================================================================== */

/* dccrg_mapping.hpp:317-330 (double arithmetic kept as in the reference) */
int dox_max_possible_refinement_level(const uint64_t length[3])
{
    const uint64_t grid_length = length[0] * length[1] * length[2];
    int refinement_level = 0;
    double current_last = 0;
    while (current_last <= (double)(~(uint64_t)0)) {
        current_last += (double)grid_length * pow(8.0, (double)refinement_level);
        refinement_level++;
    }
    return refinement_level - 2;
}

/* dccrg_mapping.hpp:679-687 */
static void update_last_cell(dox_mapping* m)
{
    const uint64_t grid_length = m->length[0] * m->length[1] * m->length[2];
    m->last_cell = 0;
    for (int i = 0; i <= m->max_ref_lvl; i++)
        m->last_cell += grid_length * ((uint64_t)1 << (i * 3));
}

/* Grid_Length::set (dccrg_length.hpp:95-130) + Mapping::set_maximum_refinement_level
 * (dccrg_mapping.hpp:135-143); returns 0 on success. */
int dox_mapping_init(dox_mapping* m, const uint64_t length[3], int32_t max_ref_lvl)
{
    if (length[0] == 0 || length[1] == 0 || length[2] == 0) return -1;
    memcpy(m->length, length, sizeof(m->length));
    m->pad_ = 0;
    if (max_ref_lvl < 0) max_ref_lvl = dox_max_possible_refinement_level(length);
    if (max_ref_lvl > dox_max_possible_refinement_level(length)) return -1;
    m->max_ref_lvl = max_ref_lvl;
    update_last_cell(m);
    return 0;
}

/* dccrg_mapping.hpp:154-209 */
uint64_t dox_get_cell_from_indices(const dox_mapping* m, const uint64_t idx[3], int lvl)
{
    const int M = m->max_ref_lvl;
    if (idx[0] >= m->length[0] * ((uint64_t)1 << M)) return DOX_ERROR_CELL;
    if (idx[1] >= m->length[1] * ((uint64_t)1 << M)) return DOX_ERROR_CELL;
    if (idx[2] >= m->length[2] * ((uint64_t)1 << M)) return DOX_ERROR_CELL;
    if (lvl < 0) return DOX_ERROR_CELL;
    if (lvl > M) return DOX_ERROR_CELL;

    uint64_t cell = 1;
    for (int i = 0; i < lvl; i++)
        cell += m->length[0] * m->length[1] * m->length[2] * ((uint64_t)1 << (i * 3));

    const uint64_t li[3] = {
        idx[0] / ((uint64_t)1 << (M - lvl)),
        idx[1] / ((uint64_t)1 << (M - lvl)),
        idx[2] / ((uint64_t)1 << (M - lvl)),
    };
    const uint64_t ll[2] = {
        m->length[0] * ((uint64_t)1 << lvl),
        m->length[1] * ((uint64_t)1 << lvl),
    };
    cell += li[0] + li[1] * ll[0] + li[2] * ll[0] * ll[1];
    return cell;
}

/* dccrg_mapping.hpp:262-290 */
int dox_get_refinement_level(const dox_mapping* m, uint64_t cell)
{
    if (cell == DOX_ERROR_CELL || cell > m->last_cell) return -1;
    int refinement_level = 0;
    uint64_t current_last = 0;
    while (refinement_level <= m->max_ref_lvl) {
        current_last += m->length[0] * m->length[1] * m->length[2]
                        * ((uint64_t)1 << 3 * refinement_level);
        if (cell <= current_last) break;
        refinement_level++;
    }
    if (refinement_level > m->max_ref_lvl) return -1;
    return refinement_level;
}

/* dccrg_mapping.hpp:218-254 */
void dox_get_indices(const dox_mapping* m, uint64_t cell, uint64_t out[3])
{
    if (cell == DOX_ERROR_CELL || cell > m->last_cell) {
        out[0] = out[1] = out[2] = DOX_ERROR_INDEX;
        return;
    }
    const int lvl = dox_get_refinement_level(m, cell);
    const int M = m->max_ref_lvl;
    for (int i = 0; i < lvl; i++)
        cell -= m->length[0] * m->length[1] * m->length[2] * ((uint64_t)1 << (i * 3));
    cell -= 1;
    out[0] = (cell % (m->length[0] * ((uint64_t)1 << lvl))) * ((uint64_t)1 << (M - lvl));
    out[1] = ((cell / (m->length[0] * ((uint64_t)1 << lvl))) % (m->length[1] * ((uint64_t)1 << lvl)))
             * ((uint64_t)1 << (M - lvl));
    out[2] = (cell / (m->length[0] * m->length[1] * ((uint64_t)1 << (2 * lvl))))
             * ((uint64_t)1 << (M - lvl));
}

/* dccrg_mapping.hpp:298-311 */
uint64_t dox_get_cell_length_in_indices(const dox_mapping* m, uint64_t cell)
{
    if (cell == DOX_ERROR_CELL) return DOX_ERROR_INDEX;
    const int lvl = dox_get_refinement_level(m, cell);
    if (lvl < 0) return DOX_ERROR_INDEX;
    return (uint64_t)1 << (m->max_ref_lvl - lvl);
}

/* dccrg_mapping.hpp:339-356 */
uint64_t dox_get_child(const dox_mapping* m, uint64_t cell)
{
    if (cell == DOX_ERROR_CELL || cell > m->last_cell) return DOX_ERROR_CELL;
    const int lvl = dox_get_refinement_level(m, cell);
    if (lvl >= m->max_ref_lvl) return cell;
    uint64_t idx[3];
    dox_get_indices(m, cell, idx);
    return dox_get_cell_from_indices(m, idx, lvl + 1);
}

/* dccrg_mapping.hpp:368-384 */
uint64_t dox_get_parent(const dox_mapping* m, uint64_t cell)
{
    const int lvl = dox_get_refinement_level(m, cell);
    if (lvl < 0 || lvl > m->max_ref_lvl) return DOX_ERROR_CELL;
    if (lvl == 0) return cell;
    uint64_t idx[3];
    dox_get_indices(m, cell, idx);
    return dox_get_cell_from_indices(m, idx, lvl - 1);
}

/* dccrg_mapping.hpp:480-494 */
uint64_t dox_get_level_0_parent(const dox_mapping* m, uint64_t cell)
{
    const int lvl = dox_get_refinement_level(m, cell);
    if (lvl < 0 || lvl > m->max_ref_lvl) return DOX_ERROR_CELL;
    if (lvl == 0) return cell;
    uint64_t idx[3];
    dox_get_indices(m, cell, idx);
    return dox_get_cell_from_indices(m, idx, 0);
}

/* dccrg_mapping.hpp:392-442 (x fastest, then y, then z) */
void dox_get_all_children(const dox_mapping* m, uint64_t cell, uint64_t out[8])
{
    for (int i = 0; i < 8; i++) out[i] = DOX_ERROR_CELL;
    if (cell == DOX_ERROR_CELL) return;
    int lvl = dox_get_refinement_level(m, cell);
    if (lvl >= m->max_ref_lvl) return;
    uint64_t idx[3];
    dox_get_indices(m, cell, idx);
    lvl++;
    const uint64_t off = (uint64_t)1 << (m->max_ref_lvl - lvl);
    size_t i = 0;
    for (uint64_t z = 0; z < 2 * off; z += off)
        for (uint64_t y = 0; y < 2 * off; y += off)
            for (uint64_t x = 0; x < 2 * off; x += off) {
                const uint64_t c[3] = {idx[0] + x, idx[1] + y, idx[2] + z};
                out[i++] = dox_get_cell_from_indices(m, c, lvl);
            }
}

/* dccrg_mapping.hpp:450-471 */
void dox_get_siblings(const dox_mapping* m, uint64_t cell, uint64_t out[8])
{
    const int lvl = dox_get_refinement_level(m, cell);
    for (int i = 0; i < 8; i++) out[i] = DOX_ERROR_CELL;
    if (lvl < 0 || lvl > m->max_ref_lvl) return;
    if (lvl == 0) {
        out[0] = cell;
        return;
    }
    dox_get_all_children(m, dox_get_parent(m, cell), out);
}

void dox_map_ids_to_indices(const dox_mapping* m, const uint64_t* ids, size_t n, uint64_t* idx3,
                            int32_t* lvl)
{
    for (size_t i = 0; i < n; i++) {
        dox_get_indices(m, ids[i], idx3 + 3 * i);
        lvl[i] = dox_get_refinement_level(m, ids[i]);
    }
}

void dox_map_indices_to_ids(const dox_mapping* m, const uint64_t* idx3, const int32_t* lvl,
                            size_t n, uint64_t* ids)
{
    for (size_t i = 0; i < n; i++) ids[i] = dox_get_cell_from_indices(m, idx3 + 3 * i, lvl[i]);
}

/* ========================================================================
 * Neighborhoods -- dccrg.hpp:8017-8076
 * ====================================================================== */
size_t dox_default_neighborhood(unsigned hood_length, int32_t* items)
{
    size_t n = 0;
    if (hood_length == 0) {
        static const int32_t face[6][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0},
                                           {1, 0, 0},  {0, 1, 0},  {0, 0, 1}};
        for (int i = 0; i < 6; i++) {
            items[3 * n + 0] = face[i][0];
            items[3 * n + 1] = face[i][1];
            items[3 * n + 2] = face[i][2];
            n++;
        }
        return n;
    }
    const int h = (int)hood_length;
    for (int z = -h; abs(z) < h + 1; z++)
        for (int y = -h; abs(y) < h + 1; y++)
            for (int x = -h; abs(x) < h + 1; x++) {
                if (x == 0 && y == 0 && z == 0) continue;
                items[3 * n + 0] = x;
                items[3 * n + 1] = y;
                items[3 * n + 2] = z;
                n++;
            }
    return n;
}

/* ========================================================================
 * Initial partition -- dccrg.hpp:8098-8145 (non-SFC)
 * ====================================================================== */
static uint64_t cells_per_process_(uint64_t total, uint64_t comm_size)
{
    if (total < comm_size) return 1;
    if (total % comm_size > 0) return total / comm_size + 1;
    return total / comm_size;
}

uint64_t dox_block_first_cell(uint64_t total, uint64_t comm_size, uint64_t rank)
{
    const uint64_t cpp = cells_per_process_(total, comm_size);
    const uint64_t fewer = cpp * comm_size - total;
    uint64_t first = 1;
    for (uint64_t p = 0; p < rank; p++) first += (p < fewer) ? cpp - 1 : cpp;
    return first;
}

uint64_t dox_block_owner(uint64_t total, uint64_t comm_size, uint64_t cell)
{
    /* the same loop as the reference: walk processes in order */
    const uint64_t cpp = cells_per_process_(total, comm_size);
    const uint64_t fewer = cpp * comm_size - total;
    uint64_t next = 1;
    for (uint64_t p = 0; p < comm_size; p++) {
        const uint64_t n = (p < fewer) ? cpp - 1 : cpp;
        if (cell < next + n) return p;
        next += n;
    }
    return comm_size; /* invalid */
}

/* ========================================================================
 * Grid: existing-cell set (stand-in for Dccrg::cell_process keys)
 * ====================================================================== */
struct dox_grid {
    dox_mapping map;
    uint8_t periodic[3];
    int all_level0; /* implicit set: every level-0 cell exists */
    uint64_t* keys; /* open addressing, 0 = empty */
    uint64_t cap;
    uint64_t count;
    uint64_t* sorted;
};

static uint64_t mix64(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

static int cmp_u64(const void* a, const void* b)
{
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return (x > y) - (x < y);
}

dox_grid* dox_grid_create(const uint64_t length[3], int32_t max_ref_lvl, const uint8_t periodic[3],
                          const uint64_t* leaves, size_t n)
{
    dox_grid* g = (dox_grid*)calloc(1, sizeof(*g));
    if (!g) return NULL;
    if (dox_mapping_init(&g->map, length, max_ref_lvl) != 0) {
        free(g);
        return NULL;
    }
    memcpy(g->periodic, periodic, 3);
    if (!leaves) {
        g->all_level0 = 1;
        g->count = length[0] * length[1] * length[2];
        return g;
    }
    g->cap = 16;
    while (g->cap < 2 * (uint64_t)n + 16) g->cap <<= 1;
    g->keys = (uint64_t*)calloc(g->cap, sizeof(uint64_t));
    g->sorted = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++) {
        const uint64_t k = leaves[i];
        if (k == DOX_ERROR_CELL) continue;
        uint64_t h = mix64(k) & (g->cap - 1);
        while (g->keys[h] != 0 && g->keys[h] != k) h = (h + 1) & (g->cap - 1);
        if (g->keys[h] == 0) {
            g->keys[h] = k;
            g->sorted[g->count++] = k;
        }
    }
    qsort(g->sorted, g->count, sizeof(uint64_t), cmp_u64);
    return g;
}

void dox_grid_destroy(dox_grid* g)
{
    if (!g) return;
    free(g->keys);
    free(g->sorted);
    free(g);
}

int dox_grid_exists(const dox_grid* g, uint64_t k)
{
    if (k == DOX_ERROR_CELL) return 0;
    if (g->all_level0) return k <= g->count;
    uint64_t h = mix64(k) & (g->cap - 1);
    while (g->keys[h] != 0) {
        if (g->keys[h] == k) return 1;
        h = (h + 1) & (g->cap - 1);
    }
    return 0;
}

size_t dox_grid_size(const dox_grid* g) { return (size_t)g->count; }

size_t dox_grid_cells(const dox_grid* g, uint64_t* out, size_t cap)
{
    size_t n = 0;
    for (uint64_t i = 0; i < g->count && n < cap; i++) out[n++] = g->all_level0 ? i + 1 : g->sorted[i];
    return n;
}

/* dccrg.hpp:11414-11447 */
uint64_t dox_get_existing_cell(const dox_grid* g, const uint64_t idx[3], int min_lvl, int max_lvl)
{
    const dox_mapping* m = &g->map;
    for (int d = 0; d < 3; d++)
        if (idx[d] >= m->length[d] * ((uint64_t)1 << m->max_ref_lvl)) return DOX_ERROR_CELL;
    if (min_lvl > max_lvl) return DOX_ERROR_CELL;
    for (int l = max_lvl; l >= min_lvl; l--) {
        const uint64_t c = dox_get_cell_from_indices(m, idx, l);
        if (dox_grid_exists(g, c)) return c;
    }
    return DOX_ERROR_CELL;
}

/* Dccrg::get_child, dccrg.hpp:9694-9718 */
uint64_t dox_grid_get_child(const dox_grid* g, uint64_t cell)
{
    const dox_mapping* m = &g->map;
    const int lvl = dox_get_refinement_level(m, cell);
    if (lvl == m->max_ref_lvl) return dox_grid_exists(g, cell) ? cell : DOX_ERROR_CELL;
    uint64_t idx[3];
    dox_get_indices(m, cell, idx);
    const uint64_t child = dox_get_cell_from_indices(m, idx, lvl + 1);
    if (dox_grid_exists(g, child)) return child;
    if (dox_grid_exists(g, cell)) return cell;
    return DOX_ERROR_CELL;
}

/* Dccrg::update_neighbors_(cell), dccrg.hpp:9463-9597 */
void dox_update_neighbors_(const dox_grid* g, uint64_t cell, uint64_t out[6])
{
    const dox_mapping* m = &g->map;
    for (int i = 0; i < 6; i++) out[i] = DOX_ERROR_CELL;
    if (cell == DOX_ERROR_CELL || !dox_grid_exists(g, cell) || cell != dox_grid_get_child(g, cell))
        return;
    uint64_t idx[3];
    dox_get_indices(m, cell, idx);
    const uint64_t cell_length = dox_get_cell_length_in_indices(m, cell);
    uint64_t s[6][3];
    for (int i = 0; i < 6; i++) memcpy(s[i], idx, sizeof(idx));
    const int M = m->max_ref_lvl;
    for (int dir = 0; dir < 6; dir += 2) { /* negative directions */
        const int d = dir / 2;
        if (s[dir][d] == 0) {
            if (!g->periodic[d]) s[dir][d] = DOX_ERROR_INDEX;
            else s[dir][d] = m->length[d] * ((uint64_t)1 << M) - 1;
        } else {
            s[dir][d]--;
        }
    }
    for (int dir = 1; dir < 6; dir += 2) { /* positive directions */
        const int d = dir / 2;
        const uint64_t max_index = m->length[d] * ((uint64_t)1 << M) - 1;
        if (max_index < cell_length || s[dir][d] > max_index - cell_length) {
            if (!g->periodic[d]) s[dir][d] = DOX_ERROR_INDEX;
            else s[dir][d] = 0;
        } else {
            s[dir][d] += cell_length;
        }
    }
    const int lvl = dox_get_refinement_level(m, cell);
    const int lo = (lvl == 0) ? 0 : lvl - 1;
    const int hi = (lvl == M) ? M : lvl + 1;
    for (int i = 0; i < 6; i++) out[i] = dox_get_existing_cell(g, s[i], lo, hi);
}

/* get_len_int lambda, dccrg.hpp:4402-4412 */
static int len_int(const dox_mapping* m, uint64_t c) { return (int)dox_get_cell_length_in_indices(m, c); }

/* get_parent_offset lambda, dccrg.hpp:4420-4437 */
static void parent_offset(const dox_mapping* m, uint64_t c, int out[3])
{
    out[0] = out[1] = out[2] = 0;
    const uint64_t parent = dox_get_parent(m, c);
    if (parent == DOX_ERROR_CELL || parent == c) return;
    uint64_t ci[3], pi[3];
    dox_get_indices(m, c, ci);
    dox_get_indices(m, parent, pi);
    for (int d = 0; d < 3; d++) {
        if (pi[d] >= ci[d]) out[d] += (int)(pi[d] - ci[d]);
        else out[d] -= (int)(ci[d] - pi[d]);
    }
}

/* adjust_offset lambda, dccrg.hpp:4440-4551; direction = +-1..3 */
static void adjust_offset(const dox_mapping* m, int off[3], uint64_t from, uint64_t to, int direction)
{
    const int from_len = len_int(m, from), to_len = len_int(m, to);
    const int dim = abs(direction) - 1;
    const int sign = direction > 0 ? 1 : -1;
    int po[3];
    if (from_len == to_len) {
        off[dim] += sign * from_len;
        return;
    }
    if (from_len < to_len) {
        parent_offset(m, from, po);
        for (int d = 0; d < 3; d++) off[d] += po[d];
        off[dim] += sign * to_len;
    } else {
        parent_offset(m, to, po);
        for (int d = 0; d < 3; d++) off[d] -= po[d];
        off[dim] += sign * from_len;
    }
}

/* Dccrg::find_neighbors_of, dccrg.hpp:4375-4716 (face-graph walk) */
long dox_find_neighbors_of(const dox_grid* g, uint64_t cell, const int32_t* items, size_t nitems,
                           uint64_t* out_ids, int32_t* out_off, size_t cap)
{
    const dox_mapping* m = &g->map;
    if (cell == DOX_ERROR_CELL || !dox_grid_exists(g, cell)) return -1;
    const int cell_length = len_int(m, cell);
    size_t n = 0;
#define PUSH(id_, x_, y_, z_)                                                                      \
    do {                                                                                           \
        if (n >= cap) return -2;                                                                   \
        out_ids[n] = (id_);                                                                        \
        out_off[3 * n + 0] = (x_);                                                                 \
        out_off[3 * n + 1] = (y_);                                                                 \
        out_off[3 * n + 2] = (z_);                                                                 \
        n++;                                                                                       \
    } while (0)

    for (size_t it = 0; it < nitems; it++) {
        const int32_t* hood = items + 3 * it;
        int os[3], oe[3];
        for (int d = 0; d < 3; d++) {
            os[d] = hood[d] * cell_length;
            oe[d] = (hood[d] + 1) * cell_length - 1;
        }
        int off[3] = {0, 0, 0};
        uint64_t current = cell;
        int cl = len_int(m, current);
        int guard = 0;
        while (off[0] + cl - 1 < os[0] || off[0] > oe[0] || off[1] + cl - 1 < os[1] ||
               off[1] > oe[1] || off[2] + cl - 1 < os[2] || off[2] > oe[2]) {
            if (++guard > 1 << 20) return -3;
            uint64_t ng[6];
            dox_update_neighbors_(g, current, ng);
            int dir_i = -1;
            if (off[0] > oe[0]) dir_i = 0;
            else if (off[0] + cl - 1 < os[0]) dir_i = 1;
            else if (off[1] > oe[1]) dir_i = 2;
            else if (off[1] + cl - 1 < os[1]) dir_i = 3;
            else if (off[2] > oe[2]) dir_i = 4;
            else if (off[2] + cl - 1 < os[2]) dir_i = 5;
            else return -4; /* internal error, dccrg.hpp:4636 */
            const int direction = (dir_i / 2 + 1) * ((dir_i % 2) ? +1 : -1);
            if (ng[dir_i] != DOX_ERROR_CELL) adjust_offset(m, off, current, ng[dir_i], direction);
            current = ng[dir_i];
            if (current == DOX_ERROR_CELL) break;
            cl = len_int(m, current);
        }
        if (current == DOX_ERROR_CELL) continue;
        cl = len_int(m, current);
        if (cl >= cell_length) {
            PUSH(current, off[0], off[1], off[2]);
            continue;
        }
        /* smaller neighbor: add all siblings, dccrg.hpp:4679-4712 */
        uint64_t sib[8];
        dox_get_siblings(m, current, sib);
        size_t ci = 0;
        for (; ci < 8; ci++)
            if (current == sib[ci]) break;
        if (ci >= 8) return -5;
        if (ci % 2 > 0) off[0] -= cl;
        if (ci % 4 > 1) off[1] -= cl;
        if (ci > 3) off[2] -= cl;
        size_t i = 0;
        for (int bz = 0; bz < 2; bz++)
            for (int by = 0; by < 2; by++)
                for (int bx = 0; bx < 2; bx++) {
                    PUSH(sib[i], off[0] + bx * cl, off[1] + by * cl, off[2] + bz * cl);
                    i++;
                }
    }
#undef PUSH
    return (long)n;
}

/* Dccrg::indices_from_neighborhood, dccrg.hpp:4236-4352 (one item) */
static void index_from_item(const dox_grid* g, const uint64_t idx[3], uint64_t len,
                            const int32_t* off, uint64_t out[3])
{
    const dox_mapping* m = &g->map;
    uint64_t G[3];
    for (int d = 0; d < 3; d++) G[d] = m->length[d] * ((uint64_t)1 << m->max_ref_lvl);
    uint64_t t[3] = {idx[0], idx[1], idx[2]};
    for (int d = 0; d < 3; d++) {
        if (off[d] < 0) {
            if (g->periodic[d]) {
                for (int i = 0; i > off[d]; i--) {
                    if (t[d] >= len) t[d] -= len;
                    else t[d] = G[d] - len;
                }
            } else {
                if (idx[d] < (uint64_t)abs(off[d]) * len) {
                    t[0] = t[1] = t[2] = DOX_ERROR_INDEX;
                    break;
                }
                t[d] += (uint64_t)(int64_t)off[d] * len;
            }
        } else {
            if (g->periodic[d]) {
                for (int i = 0; i < off[d]; i++) {
                    if (t[d] < G[d] - len) t[d] += len;
                    else t[d] = 0;
                }
            } else {
                if (idx[d] + (uint64_t)off[d] * len >= G[d]) {
                    t[0] = t[1] = t[2] = DOX_ERROR_INDEX;
                    break;
                }
                t[d] += (uint64_t)off[d] * len;
            }
        }
    }
    memcpy(out, t, sizeof(t));
}

static size_t uniq_sorted(uint64_t* v, size_t n)
{
    if (n == 0) return 0;
    qsort(v, n, sizeof(uint64_t), cmp_u64);
    size_t w = 1;
    for (size_t i = 1; i < n; i++)
        if (v[i] != v[w - 1]) v[w++] = v[i];
    return w;
}

/* Dccrg::find_neighbors_to, dccrg.hpp:4744-4897.  The reference returns
 * unordered_map order; this restatement returns ascending ids. */
long dox_find_neighbors_to(const dox_grid* g, uint64_t cell, const int32_t* items, size_t nitems,
                           uint64_t* out_ids, size_t cap)
{
    const dox_mapping* m = &g->map;
    if (cell == DOX_ERROR_CELL || cell > m->last_cell || cell != dox_grid_get_child(g, cell))
        return -1;
    const int lvl = dox_get_refinement_level(m, cell);
    size_t tmp_cap = nitems * 10 + 8;
    uint64_t* tmp = (uint64_t*)malloc(tmp_cap * sizeof(uint64_t));
    size_t n = 0;
    uint64_t s[3], idx[3];
    if (lvl > 0) {
        const uint64_t parent = dox_get_parent(m, cell);
        dox_get_indices(m, parent, idx);
        const uint64_t len = dox_get_cell_length_in_indices(m, parent);
        for (size_t i = 0; i < nitems; i++) {
            index_from_item(g, idx, len, items + 3 * i, s);
            if (s[0] == DOX_ERROR_INDEX) continue;
            const uint64_t found = dox_get_cell_from_indices(m, s, lvl - 1);
            if (found == dox_grid_get_child(g, found)) tmp[n++] = found;
        }
    }
    if (lvl < m->max_ref_lvl) {
        uint64_t ch[8];
        dox_get_all_children(m, cell, ch);
        const uint64_t len = dox_get_cell_length_in_indices(m, ch[0]);
        for (int c = 0; c < 8; c++) {
            dox_get_indices(m, ch[c], idx);
            for (size_t i = 0; i < nitems; i++) {
                index_from_item(g, idx, len, items + 3 * i, s);
                if (s[0] == DOX_ERROR_INDEX) continue;
                const uint64_t found = dox_get_cell_from_indices(m, s, lvl + 1);
                if (found == dox_grid_get_child(g, found)) tmp[n++] = found;
            }
        }
    }
    dox_get_indices(m, cell, idx);
    const uint64_t len = dox_get_cell_length_in_indices(m, cell);
    for (size_t i = 0; i < nitems; i++) {
        index_from_item(g, idx, len, items + 3 * i, s);
        if (s[0] == DOX_ERROR_INDEX) continue;
        const uint64_t found = dox_get_cell_from_indices(m, s, lvl);
        if (found == dox_grid_get_child(g, found)) tmp[n++] = found;
    }
    n = uniq_sorted(tmp, n);
    if (n > cap) {
        free(tmp);
        return -2;
    }
    memcpy(out_ids, tmp, n * sizeof(uint64_t));
    free(tmp);
    return (long)n;
}

/* Dccrg::get_face_neighbors_of, dccrg.hpp:2828-2955 */
long dox_get_face_neighbors_of(const dox_grid* g, uint64_t cell, uint64_t* out_ids, int32_t* out_dirs,
                               size_t cap)
{
    const dox_mapping* m = &g->map;
    if (!dox_grid_exists(g, cell)) return -1;
    static const int dirs[6] = {-1, +1, -2, +2, -3, +3};
    uint64_t ng[6];
    dox_update_neighbors_(g, cell, ng);
    const int lvl = dox_get_refinement_level(m, cell);
    size_t n = 0;
#define PUSHF(id_, d_)                                                                             \
    do {                                                                                           \
        if (n >= cap) return -2;                                                                   \
        out_ids[n] = (id_);                                                                        \
        out_dirs[n] = (d_);                                                                        \
        n++;                                                                                       \
    } while (0)
    for (int i = 0; i < 6; i++) {
        const uint64_t nb = ng[i];
        if (nb == DOX_ERROR_CELL) continue;
        PUSHF(nb, dirs[i]);
        if (lvl >= dox_get_refinement_level(m, nb)) continue;
        uint64_t nn[6], nnn[6];
        dox_update_neighbors_(g, nb, nn);
        int a, b; /* the two tangential positive directions */
        if (i < 2) { a = 3; b = 5; }
        else if (i < 4) { a = 1; b = 5; }
        else { a = 1; b = 3; }
        if (nn[a] != DOX_ERROR_CELL) PUSHF(nn[a], dirs[i]);
        if (nn[b] != DOX_ERROR_CELL) {
            PUSHF(nn[b], dirs[i]);
            dox_update_neighbors_(g, nn[b], nnn);
            if (nnn[a] != DOX_ERROR_CELL) PUSHF(nnn[a], dirs[i]);
        }
    }
#undef PUSHF
    return (long)n;
}

/* ========================================================================
 * Game of life over explicit lists -- the reference's user hot loop
 * ====================================================================== */
void dox_gol_count(size_t n_cells, const uint64_t* row_ptr, const uint32_t* nbr_slot,
                   const uint32_t* alive, uint32_t* count)
{
    /* examples/game_of_life.cpp:54-66: live_neighbor_count = #alive neighbors_of
     * (cells are independent: host threads split them, results unchanged) */
#pragma omp parallel for schedule(static)
    for (size_t c = 0; c < n_cells; c++) {
        uint32_t cnt = 0;
        for (uint64_t k = row_ptr[c]; k < row_ptr[c + 1]; k++)
            if (alive[nbr_slot[k]] > 0) cnt++;
        count[c] = cnt;
    }
}

void dox_gol_apply(size_t n_cells, uint32_t* alive, const uint32_t* count)
{
    /* examples/game_of_life.cpp:68-79 (B3/S23) */
#pragma omp parallel for schedule(static)
    for (size_t c = 0; c < n_cells; c++) {
        if (count[c] == 3) alive[c] = 1;
        else if (count[c] != 2) alive[c] = 0;
    }
}

int dox_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* the thread count of the parallel loops (the CPU baseline's sweep) */
void dox_set_num_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

long dox_build_uniform_slot_lists(const dox_grid* g, unsigned hood_length, uint64_t* row_ptr,
                                  uint32_t* nbr_slot, size_t cap)
{
    int32_t items[3 * 343];
    const size_t ni = dox_default_neighborhood(hood_length, items);
    uint64_t* ids = (uint64_t*)malloc(8 * ni * sizeof(uint64_t));
    int32_t* off = (int32_t*)malloc(8 * ni * 3 * sizeof(int32_t));
    size_t n = 0;
    row_ptr[0] = 0;
    for (uint64_t c = 1; c <= g->count; c++) {
        const long k = dox_find_neighbors_of(g, c, items, ni, ids, off, 8 * ni);
        if (k < 0 || n + (size_t)k > cap) {
            free(ids);
            free(off);
            return -1;
        }
        for (long j = 0; j < k; j++) nbr_slot[n++] = (uint32_t)(ids[j] - 1);
        row_ptr[c] = n;
    }
    free(ids);
    free(off);
    return (long)n;
}

/* ---- Advection (tests/advection/solve.hpp) ---------------------------- */

/* calculate_fluxes, solve.hpp:44-247, for the cells iter_slot[0..n_iter),
 * each with its iteration-cache neighbors_of row (slots + offsets).  Face
 * detection :73-120, local pairs solved once in the positive direction
 * :125-128, min_area :134-157, interpolated velocity :165-171, upwind flux
 * :173-221, accumulation into BOTH cells :224-230 (into ghost copies too;
 * the reference discards those).  Returns the number of overlaps > 2 pairs
 * (the reference aborts, :101-116). */
long dox_advect_fluxes(size_t n_iter, const uint32_t* iter_slot, const uint64_t* row_ptr,
                       const uint32_t* nbr_slot, const int32_t* nbr_off, const uint8_t* is_local,
                       const uint64_t* len_idx, const double* density, const double* vx,
                       const double* vy, const double* vz, const double* lx, const double* ly,
                       const double* lz, double* flux, double dt)
{
    long bad = 0;
    for (size_t i = 0; i < n_iter; i++) {
        const uint32_t c = iter_slot[i];
        const double cell_density = density[c], cell_volume = lx[c] * ly[c] * lz[c];
        const int64_t cl = (int64_t)len_idx[c];
        for (uint64_t e = row_ptr[i]; e < row_ptr[i + 1]; e++) {
            const uint32_t nb = nbr_slot[e];
            const int64_t nl = (int64_t)len_idx[nb];
            int overlaps = 0, direction = 0;
            for (int d = 0; d < 3; d++) {
                const int64_t o = nbr_off[3 * e + d];
                if (o < cl && o > -nl) overlaps++;
                else if (o == cl) direction = d + 1;
                else if (o == -nl) direction = -(d + 1);
            }
            if (overlaps < 2) continue;
            if (overlaps > 2) {
                bad++;
                continue;
            }
            if (direction == 0) continue;
            if (is_local[nb] && direction < 0) continue;
            const double neighbor_density = density[nb], neighbor_volume = lx[nb] * ly[nb] * lz[nb];
            double min_area = -1;
            switch (direction) {
            case -1: case 1: {
                const double a = ly[c] * lz[c], b = ly[nb] * lz[nb];
                min_area = a < b ? a : b;
                break;
            }
            case -2: case 2: {
                const double a = lx[c] * lz[c], b = lx[nb] * lz[nb];
                min_area = a < b ? a : b;
                break;
            }
            default: {
                const double a = lx[c] * ly[c], b = lx[nb] * ly[nb];
                min_area = a < b ? a : b;
                break;
            }
            }
            const double v_x = (lx[c] * vx[nb] + lx[nb] * vx[c]) / (lx[c] + lx[nb]);
            const double v_y = (ly[c] * vy[nb] + ly[nb] * vy[c]) / (ly[c] + ly[nb]);
            const double v_z = (lz[c] * vz[nb] + lz[nb] * vz[c]) / (lz[c] + lz[nb]);
            const double v = direction == 1 || direction == -1 ? v_x : direction == 2 || direction == -2 ? v_y : v_z;
            double f;
            if (direction > 0) f = (v >= 0 ? cell_density : neighbor_density) * dt * v * min_area;
            else f = (v >= 0 ? neighbor_density : cell_density) * dt * v * min_area;
            if (direction > 0) {
                flux[c] -= f / cell_volume;
                flux[nb] += f / neighbor_volume;
            } else {
                flux[c] += f / cell_volume;
                flux[nb] -= f / neighbor_volume;
            }
        }
    }
    return bad;
}

/* apply_fluxes, solve.hpp:283-293 */
void dox_advect_apply(size_t n, const uint32_t* slot, double* density, double* flux)
{
    for (size_t i = 0; i < n; i++) {
        density[slot[i]] += flux[slot[i]];
        flux[slot[i]] = 0;
    }
}

/* max_time_step, solve.hpp:302-332, local part (before MPI_Allreduce MIN) */
double dox_advect_max_time_step(size_t n, const uint32_t* slot, const double* vx, const double* vy,
                                const double* vz, const double* lx, const double* ly, const double* lz)
{
    double m = DBL_MAX;
    for (size_t i = 0; i < n; i++) {
        const uint32_t c = slot[i];
        const double s[3] = {lx[c] / fabs(vx[c]), ly[c] / fabs(vy[c]), lz[c] / fabs(vz[c])};
        for (int d = 0; d < 3; d++)
            if (isnormal(s[d]) && s[d] < m) m = s[d];
    }
    return m;
}

/* ---- Poisson, tests/poisson/poisson_solve.hpp ------------------------- */

/* multiplier of a cell's own factor for a neighbor in direction dir (and the
 * transposed one, taken from the neighbor), poisson_solve.hpp:290-330,
 * :430-470; f holds f_x_pos, f_x_neg, f_y_pos, f_y_neg, f_z_pos, f_z_neg */
static int pf_index(int dir) { return dir > 0 ? 2 * (dir - 1) : 2 * (-dir - 1) + 1; }

/* Poisson_Solve::solve iterations (poisson_solve.hpp:251-522) and
 * initialize_solver (:976-1056) over the cached cell_info (:892-971).  Rank
 * r's cell_info entries are [rank_begin[r], rank_begin[r+1]); per-rank
 * partial sums are added in rank order (MPI_Allreduce SUM).  Ghost copies
 * are the owners' values (every read happens right after the exchange the
 * reference does).  nb_code = (dir + 3) | ((rel + 1) << 4). */
long dox_poisson_solve(size_t n_info, const uint32_t* info_slot, int P, const size_t* rank_begin,
                       const uint64_t* row, const uint32_t* nb_slot, const int32_t* nb_code,
                       const double* type, const double* rhs, double* solution, double* best,
                       double* p0, double* p1, double* r0, double* r1, double* adp0, const double* sf,
                       const double* f /* 6 per slot */, unsigned max_iterations, unsigned min_iterations,
                       double stop_residual, double p_of_norm, double stop_after_residual_increase,
                       double* residual_min_out)
{
    double part[256];
    if (P > 256) return -1;
#define ALLREDUCE(expr_, cond_, out_)                                                            \
    do {                                                                                         \
        double tot_ = 0;                                                                         \
        for (int r_ = 0; r_ < P; r_++) {                                                         \
            part[r_] = 0;                                                                        \
            for (size_t i = rank_begin[r_]; i < rank_begin[r_ + 1]; i++) {                       \
                const uint32_t c = info_slot[i];                                                 \
                (void)c;                                                                         \
                if (cond_) part[r_] += (expr_);                                                  \
            }                                                                                    \
        }                                                                                        \
        for (int r_ = 0; r_ < P; r_++) tot_ += part[r_];                                         \
        out_ = tot_;                                                                             \
    } while (0)
    /* initialize_solver: r0 = rhs - A . solution; p0 = p1 = r1 = r0 */
    for (size_t i = 0; i < n_info; i++) {
        const uint32_t c = info_slot[i];
        if (type[c] != 0) continue;
        r0[c] = rhs[c] - sf[c] * solution[c];
        for (uint64_t e = row[i]; e < row[i + 1]; e++) {
            const int dir = (nb_code[e] & 15) - 3, rel = (nb_code[e] >> 4) - 1;
            double m = f[6 * c + pf_index(dir)];
            if (rel > 0) m /= 4.0;
            r0[c] -= m * solution[nb_slot[e]];
        }
        p0[c] = p1[c] = r1[c] = r0[c];
    }
    double dot_r_g;
    ALLREDUCE(r0[c] * r1[c], type[c] == 0, dot_r_g);
    double residual_min = DBL_MAX;
    size_t iteration = 0;
    do {
        iteration++;
        for (size_t i = 0; i < n_info; i++) {  /* A . p0 */
            const uint32_t c = info_slot[i];
            if (type[c] != 0) continue;
            adp0[c] = sf[c] * p0[c];
            for (uint64_t e = row[i]; e < row[i + 1]; e++) {
                const int dir = (nb_code[e] & 15) - 3, rel = (nb_code[e] >> 4) - 1;
                double m = f[6 * c + pf_index(dir)];
                if (rel > 0) m /= 4.0;
                adp0[c] += m * p0[nb_slot[e]];
            }
        }
        double dot_p_g;
        ALLREDUCE(p1[c] * adp0[c], type[c] == 0, dot_p_g);
        if (dot_p_g == 0) break;
        const double alpha = dot_r_g / dot_p_g;
        for (size_t i = 0; i < n_info; i++) {
            const uint32_t c = info_slot[i];
            if (type[c] == 0) solution[c] += alpha * p0[c];
        }
        double residual; /* get_residual, :684-697 (all cell_info cells) */
        ALLREDUCE(pow(fabs(r0[c]), p_of_norm), 1, residual);
        residual = pow(residual, 1.0 / p_of_norm);
        if (residual_min > residual) {
            residual_min = residual;
            for (size_t i = 0; i < n_info; i++) {
                const uint32_t c = info_slot[i];
                if (type[c] == 0) best[c] = solution[c];
            }
        }
        if (residual <= stop_residual && iteration >= min_iterations) break;
        if (residual >= stop_after_residual_increase * residual_min && iteration >= min_iterations) break;
        for (size_t i = 0; i < n_info; i++) {
            const uint32_t c = info_slot[i];
            if (type[c] == 0) r0[c] -= alpha * adp0[c];
        }
        for (size_t i = 0; i < n_info; i++) {  /* r1 -= alpha * transpose(A) . p1 */
            const uint32_t c = info_slot[i];
            if (type[c] != 0) continue;
            double a = sf[c] * p1[c];
            for (uint64_t e = row[i]; e < row[i + 1]; e++) {
                const int dir = (nb_code[e] & 15) - 3, rel = (nb_code[e] >> 4) - 1;
                const uint32_t nb = nb_slot[e];
                double m = f[6 * nb + pf_index(-dir)];
                if (rel > 0) m /= 4.0;
                a += m * p1[nb];
            }
            r1[c] -= alpha * a;
        }
        if (dot_r_g == 0) break;
        const double old = dot_r_g;
        ALLREDUCE(r0[c] * r1[c], type[c] == 0, dot_r_g);
        const double beta = dot_r_g / old;
        for (size_t i = 0; i < n_info; i++) {
            const uint32_t c = info_slot[i];
            if (type[c] == 0) {
                p0[c] = r0[c] + beta * p0[c];
                p1[c] = r1[c] + beta * p1[c];
            }
        }
    } while (iteration < max_iterations);
#undef ALLREDUCE
    for (size_t i = 0; i < n_info; i++) {
        const uint32_t c = info_slot[i];
        if (type[c] == 0) solution[c] = best[c];
    }
    *residual_min_out = residual_min;
    return (long)iteration;
}
