/* TEST INFRASTRUCTURE ONLY.  The reference's own advection solver
 * (tests/advection/solve.hpp, adapter.hpp, initialize.hpp, cell.hpp, compiled
 * where they lie under /root/reference) driven the way tests/advection/2d.cpp
 * drives it with its default options (:250-440: balance_load, pre-refinement,
 * then per step start updates, inner fluxes, wait, outer fluxes,
 * check_for_adaptation, apply_fluxes, adapt_grid, max_time_step, balance_load
 * every 25 steps), over this repository's drop-in dccrg::Dccrg
 * (include/dccrg.hpp -> include/dccrg_amd.hpp).  The solver arithmetic, the
 * adaptation rules and the data rules of new and removed cells are the
 * reference's source; the grid underneath (lists, refinement, host data) is
 * ours.  Built by `make -C oracle ref` into oracle/_ref/; run on the GPU box by
 * tests/test_gpu_ref_advection.py, which compares the device solver with it.
 *
 * argv: cells_per_side max_ref_lvl steps adapt_n out_path
 * out: per state (after pre-refinement, then after every step):
 *      u64 step, f64 dt, u64 n, n x (u64 id, f64 density), ids ascending
 */
#include <mpi.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <tuple>
#include <unordered_set>
#include <utility>
#include <vector>

#include "dccrg.hpp"
#include "dccrg_cartesian_geometry.hpp"

#include "cell.hpp"

bool Cell::transfer_all_data = false;

#include "adapter.hpp"
#include "initialize.hpp"
#include "solve.hpp"

using namespace dccrg;

typedef Dccrg<Cell, Cartesian_Geometry, std::tuple<Center>, std::tuple<Is_Local>> Grid;

static void dump(FILE* f, uint64_t step, double dt, Grid& grid)
{
    std::vector<uint64_t> ids = grid.get_cells();
    std::sort(ids.begin(), ids.end());
    const uint64_t n = ids.size();
    fwrite(&step, 8, 1, f);
    fwrite(&dt, 8, 1, f);
    fwrite(&n, 8, 1, f);
    for (uint64_t c : ids) {
        const double d = grid[c]->density();
        fwrite(&c, 8, 1, f);
        fwrite(&d, 8, 1, f);
    }
}

int main(int argc, char** argv)
{
    MPI_Init(&argc, &argv);
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s cells_per_side max_ref_lvl steps adapt_n out\n", argv[0]);
        return 1;
    }
    const uint64_t n = std::strtoull(argv[1], nullptr, 10);
    const int max_ref_lvl = std::atoi(argv[2]);
    const int steps = std::atoi(argv[3]), adapt_n = std::atoi(argv[4]);
    // 2d.cpp's defaults (:90-125): cfl 0.5, relative-diff 0.025, diff-threshold 0.25, unrefine-sensitivity 0.5
    const double cfl = 0.5, relative_diff = 0.025, diff_threshold = 0.25, unrefine_sensitivity = 0.5;
    MPI_Comm comm = MPI_COMM_WORLD;
    FILE* f = std::fopen(argv[5], "wb");
    if (!f) return 1;

    Grid grid;
    Cartesian_Geometry::Parameters geom_params;
    for (int d = 0; d < 3; d++) {
        geom_params.start[d] = 0;
        geom_params.level_0_cell_length[d] = 1.0 / n;
    }
    grid.set_neighborhood_length(0).set_maximum_refinement_level(max_ref_lvl);
    grid.set_initial_length({{n, n, 1}}).set_periodic(true, true, false);
    grid.initialize(comm).set_geometry(geom_params);
    const int balance_n = 25;  // 2d.cpp's default (:114-115)
    grid.balance_load();       // :254-256 (DCCRG_NO_LB: a no-op)
    // the Center items were computed before set_geometry; the reference's
    // Zoltan build refreshes them in balance_load (update_cell_pointers), the
    // facade does it on request
    grid.refresh_additional_items();

    const bool dbg = std::getenv("REF_ADVECTION_DEBUG") != nullptr;
    Cell::transfer_all_data = true;
    initialize(grid);
    std::unordered_set<uint64_t> to_refine, not_to_unrefine, to_unrefine;
    for (int lvl = 0; lvl < max_ref_lvl; lvl++) {
        check_for_adaptation(relative_diff / grid.get_maximum_refinement_level(), diff_threshold, unrefine_sensitivity,
                             to_refine, not_to_unrefine, to_unrefine, grid);
        if (dbg) {
            double mass = 0, cx = 0;
            for (const auto& cell : grid.local_cells()) {
                mass += cell.data->density();
                cx += cell.center[0];
            }
            std::fprintf(stderr, "pre-refine %d: cells %zu mass %.17g sum_cx %.17g refine %zu keep %zu unrefine %zu\n",
                         lvl, grid.get_cells().size(), mass, cx, to_refine.size(), not_to_unrefine.size(),
                         to_unrefine.size());
        }
        const auto ad = adapt_grid(to_refine, not_to_unrefine, to_unrefine, grid);
        if (dbg)
            std::fprintf(stderr, "  adapt_grid created %llu removed %llu -> cells %zu\n", (unsigned long long)ad.first,
                         (unsigned long long)ad.second, grid.get_cells().size());
        initialize(grid);
    }
    Cell::transfer_all_data = false;
    double dt = max_time_step(comm, grid);
    dump(f, 0, dt, grid);

    for (int step = 0; step < steps; step++) {
        grid.start_remote_neighbor_copy_updates();
        calculate_fluxes(cfl * dt, true, grid);
        grid.wait_remote_neighbor_copy_update_receives();
        calculate_fluxes(cfl * dt, false, grid);
        grid.wait_remote_neighbor_copy_update_sends();
        const bool adapt = adapt_n > 0 && step % adapt_n == 0;
        if (adapt)
            check_for_adaptation(relative_diff / grid.get_maximum_refinement_level(), diff_threshold,
                                 unrefine_sensitivity, to_refine, not_to_unrefine, to_unrefine, grid);
        apply_fluxes(grid);
        if (adapt) {
            Cell::transfer_all_data = true;
            adapt_grid(to_refine, not_to_unrefine, to_unrefine, grid);
            Cell::transfer_all_data = false;
            dt = max_time_step(comm, grid);
        }
        if (balance_n > 0 && step % balance_n == 0) {  // :422-434
            Cell::transfer_all_data = true;
            grid.balance_load();
            grid.update_copies_of_remote_neighbors();
            Cell::transfer_all_data = false;
        }
        dump(f, (uint64_t)step + 1, dt, grid);
    }
    std::fclose(f);
    MPI_Finalize();
    return 0;
}
