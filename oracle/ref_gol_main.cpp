/* TEST INFRASTRUCTURE ONLY.  The reference's own AMR-aware game of life
 * (tests/game_of_life/solve.hpp get_live_neighbors + cell.hpp, compiled where
 * they lie under /root/reference) over this repository's drop-in dccrg.hpp,
 * driven as game_of_life_test.cpp / refined2d.cpp drive it (:378-414: update
 * the ghosts, then get_live_neighbors).  Built by `make -C oracle ref` into
 * oracle/_ref/; run on the GPU box by tests/test_gpu_ref_gol.py, which
 * compares the device kernels (golh.hip) with it.
 *
 * argv: Lx Ly refine_permille seed steps out_path
 * The grid: Lx x Ly x 1, periodic x and y, neighborhood length 1, maximum
 * refinement level 1; level-0 cells with splitmix64(id ^ seed) % 1000 <
 * refine_permille refined once; a cell is alive when splitmix64(its level-0
 * parent) % 1000 < 300, children take their parent's state.
 * out: per state (initial, then after every step): u64 step, u64 n,
 *      n x (u64 id, u64 data[0]), ids ascending
 */
#include <mpi.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dccrg.hpp"

#include "cell.hpp"
#include "solve.hpp"

using namespace dccrg;

static uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void dump(FILE* f, uint64_t step, Dccrg<Cell>& grid)
{
    std::vector<uint64_t> ids = grid.get_cells();
    std::sort(ids.begin(), ids.end());
    const uint64_t n = ids.size();
    fwrite(&step, 8, 1, f);
    fwrite(&n, 8, 1, f);
    for (uint64_t c : ids) {
        const uint64_t a = grid[c]->data[0];
        fwrite(&c, 8, 1, f);
        fwrite(&a, 8, 1, f);
    }
}

int main(int argc, char** argv)
{
    MPI_Init(&argc, &argv);
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s Lx Ly refine_permille seed steps out\n", argv[0]);
        return 1;
    }
    const uint64_t lx = std::strtoull(argv[1], nullptr, 10), ly = std::strtoull(argv[2], nullptr, 10);
    const uint64_t permille = std::strtoull(argv[3], nullptr, 10), seed = std::strtoull(argv[4], nullptr, 10);
    const int steps = std::atoi(argv[5]);
    FILE* f = std::fopen(argv[6], "wb");
    if (!f) return 1;

    Dccrg<Cell> grid;
    grid.set_initial_length({{lx, ly, 1}})
        .set_neighborhood_length(1)
        .set_maximum_refinement_level(1)
        .set_periodic(true, true, false)
        .initialize(MPI_COMM_WORLD);
    for (uint64_t c : grid.get_cells())
        if (splitmix64(c ^ seed) % 1000 < permille) grid.refine_completely(c);
    grid.stop_refining();
    grid.clear_refined_unrefined_data();
    for (uint64_t c : grid.get_cells()) {
        Cell* d = grid[c];
        for (auto& v : d->data) v = 0;
        d->data[0] = splitmix64(grid.mapping.get_level_0_parent(c)) % 1000 < 300 ? 1 : 0;
    }
    dump(f, 0, grid);
    for (int step = 0; step < steps; step++) {
        grid.update_copies_of_remote_neighbors();
        get_live_neighbors(grid);
        dump(f, (uint64_t)step + 1, grid);
    }
    std::fclose(f);
    MPI_Finalize();
    return 0;
}
