// User programs written against the dccrg interface (include/dccrg_amd.hpp),
// the way the reference's examples and tests use it.  Modes:
//   blinker          examples/simple_game_of_life.cpp semantics (aborts on error)
//   scal3d LX LY LZ STEPS PX PY PZ
//                    tests/game_of_life/scalability3d.cpp loop (start, inner,
//                    wait, outer, rule); prints "alive <id>" lines
//   halo             examples/basic_cell_data.cpp (Dccrg<int>, ghosts == ids)
//   mapping          prints Mapping results for a list of ids
//   lists            prints the iteration-cache neighbor lists of every cell
//   restart FILE     tests/restart/restart_test.cpp's property: a 15x15 game
//                    saved at step 5 (header = step), loaded into a new grid
//                    and continued equals the uninterrupted game at step 10
//   amr CELL...      refines CELLs (6x5x4, max level 1, hood 1, periodic y z),
//                    checks the data movement, prints new cells and the
//                    rebuilt iteration-cache lists; then unrefines them back
//   overlap LX LY LZ STEPS PX PY PZ
//                    examples/game_of_life.cpp:117-139's turn: one message per
//                    cell (set_send_single_cells), receives and sends started
//                    separately, inner counts, wait receives, outer counts,
//                    inner rules, wait sends, outer rules; checks
//                    get_neighbors_of_at_offset against neighbors_of; prints
//                    "alive <id> <count>" lines (any number of MPI ranks)
//   cells ...        get_cells criteria and process-boundary accessors
//   coords           geometry lookups, refinement at a coordinate, no-LB calls
//   copy             the converting copy constructor (tests/constructors/copy.cpp)
//   varneigh [LX LY] variable-size cell data in halos (variable_neighbour_data.cpp)
//   interlaced       user_neighborhood/game_of_life.cpp (4 games, hood of +-2)
//   items            additional_cell_data/*.cpp (items, grid.cells, No_Geometry)
//   nocopy           constructors/simple.cpp (cell data never copied or moved)
//   vtk PREFIX       write_vtk_file of each rank's leaves (PREFIX_<rank>.vtk)
// Built with the reference's own flags (-std=c++11, Makefile:8) by the tests.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>

#include "dccrg_amd.hpp"

struct game_of_life_cell {
    unsigned int is_alive = 0, live_neighbor_count = 0;
    std::tuple<void*, int, MPI_Datatype> get_mpi_datatype()
    {
        return std::make_tuple((void*)&(this->is_alive), 1, MPI_UNSIGNED);
    }
};

static uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int blinker()
{
    dccrg::Dccrg<game_of_life_cell> grid;
    grid.set_initial_length({10, 10, 1})
        .set_maximum_refinement_level(0)
        .set_neighborhood_length(1)
        .set_load_balancing_method("RCB")
        .initialize(MPI_COMM_WORLD);
    grid.balance_load();
    for (const auto& cell : grid.local_cells()) {
        cell.data->live_neighbor_count = 0;
        cell.data->is_alive = (cell.id == 54 || cell.id == 55 || cell.id == 56) ? 1 : 0;
    }
    for (int turn = 0; turn < 100; turn++) {
        grid.update_copies_of_remote_neighbors();
        for (const auto& cell : grid.local_cells()) {
            cell.data->live_neighbor_count = 0;
            for (const auto& neighbor : cell.neighbors_of)
                if (neighbor.data->is_alive > 0) cell.data->live_neighbor_count++;
        }
        for (const auto& cell : grid.local_cells()) {
            if (cell.data->live_neighbor_count == 3) cell.data->is_alive = 1;
            else if (cell.data->live_neighbor_count != 2) cell.data->is_alive = 0;
        }
        for (const auto& cell : grid.local_cells()) {
            const bool even = turn % 2 == 0;
            if (cell.id == 55 && !cell.data->is_alive) abort();
            if ((cell.id == 54 || cell.id == 56) && (cell.data->is_alive != (even ? 0u : 1u))) abort();
            if ((cell.id == 45 || cell.id == 65) && (cell.data->is_alive != (even ? 1u : 0u))) abort();
        }
    }
    printf("PASS blinker\n");
    return 0;
}

static int scal3d(int argc, char** argv)
{
    const uint64_t L[3] = {strtoull(argv[2], 0, 10), strtoull(argv[3], 0, 10), strtoull(argv[4], 0, 10)};
    const int steps = atoi(argv[5]);
    dccrg::Dccrg<game_of_life_cell> grid;
    grid.set_initial_length({L[0], L[1], L[2]})
        .set_neighborhood_length(1)
        .set_maximum_refinement_level(0)
        .set_periodic(atoi(argv[6]), atoi(argv[7]), atoi(argv[8]))
        .initialize(MPI_COMM_WORLD)
        .balance_load();
    for (const auto& cell : grid.local_cells()) {
        cell.data->live_neighbor_count = 0;
        cell.data->is_alive = splitmix64(cell.id) % 1000 < 200;
    }
    for (int step = 0; step < steps; step++) {
        grid.start_remote_neighbor_copy_updates();
        for (const auto& cell : grid.inner_cells()) {
            cell.data->live_neighbor_count = 0;
            for (const auto& neighbor : cell.neighbors_of)
                if (neighbor.data->is_alive) cell.data->live_neighbor_count++;
        }
        grid.wait_remote_neighbor_copy_updates();
        for (const auto& cell : grid.outer_cells()) {
            cell.data->live_neighbor_count = 0;
            for (const auto& neighbor : cell.neighbors_of)
                if (neighbor.data->is_alive) cell.data->live_neighbor_count++;
        }
        for (const auto& cell : grid.local_cells()) {
            if (cell.data->live_neighbor_count == 3) cell.data->is_alive = true;
            else if (cell.data->live_neighbor_count != 2) cell.data->is_alive = false;
        }
    }
    for (const auto& cell : grid.local_cells())
        if (cell.data->is_alive) printf("alive %llu %u\n", (unsigned long long)cell.id, cell.data->live_neighbor_count);
    return 0;
}

static int halo()
{
    dccrg::Dccrg<int> grid;
    grid.set_initial_length({7, 13, 11})
        .set_maximum_refinement_level(1)
        .set_neighborhood_length(2)
        .set_load_balancing_method("RANDOM")
        .set_periodic(true, true, true)
        .initialize(MPI_COMM_WORLD)
        .balance_load();
    for (const auto& cell : grid.local_cells()) *cell.data = (int)cell.id;
    grid.update_copies_of_remote_neighbors();
    size_t checked = 0;
    for (const auto& cell : grid.local_cells())
        for (const auto& neighbor : cell.neighbors_of) {
            if (*neighbor.data != (int)neighbor.id) abort();
            checked++;
        }
    printf("PASS halo %zu\n", checked);
    return 0;
}

static int mapping()
{
    dccrg::Dccrg<int> grid;
    grid.set_initial_length({100, 200, 300}).set_maximum_refinement_level(13);
    const auto& m = grid.mapping;
    const uint64_t ids[] = {1, 2, 100, 6000000, 6000001, 48000001, 123456789, 9000000000ull, m.get_last_cell(),
                            m.get_last_cell() + 1, 0};
    for (uint64_t id : ids) {
        const auto idx = m.get_indices(id);
        printf("%llu %d %llu %llu %llu %llu %llu %llu\n", (unsigned long long)id, m.get_refinement_level(id),
               (unsigned long long)idx[0], (unsigned long long)idx[1], (unsigned long long)idx[2],
               (unsigned long long)m.get_parent(id), (unsigned long long)m.get_level_0_parent(id),
               (unsigned long long)m.get_cell_length_in_indices(id));
    }
    return 0;
}

static int lists(int argc, char** argv)
{
    dccrg::Dccrg<int> grid;
    grid.set_initial_length({strtoull(argv[2], 0, 10), strtoull(argv[3], 0, 10), strtoull(argv[4], 0, 10)})
        .set_neighborhood_length(atoi(argv[8]))
        .set_maximum_refinement_level(0)
        .set_periodic(atoi(argv[5]), atoi(argv[6]), atoi(argv[7]))
        .initialize(MPI_COMM_WORLD);
    for (const auto& cell : grid.local_cells()) {
        printf("cell %llu of", (unsigned long long)cell.id);
        for (const auto& n : cell.neighbors_of) printf(" %llu:%d,%d,%d", (unsigned long long)n.id, n.x, n.y, n.z);
        printf(" to");
        for (const auto& n : cell.neighbors_to) printf(" %llu:%d,%d,%d", (unsigned long long)n.id, n.x, n.y, n.z);
        printf("\n");
    }
    return 0;
}

template <class Grid> static void gol_turn(Grid& grid)
{
    grid.update_copies_of_remote_neighbors();
    for (const auto& cell : grid.local_cells()) {
        cell.data->live_neighbor_count = 0;
        for (const auto& neighbor : cell.neighbors_of)
            if (neighbor.data->is_alive) cell.data->live_neighbor_count++;
    }
    for (const auto& cell : grid.local_cells()) {
        if (cell.data->live_neighbor_count == 3) cell.data->is_alive = 1;
        else if (cell.data->live_neighbor_count != 2) cell.data->is_alive = 0;
    }
}

static int restart(int argc, char** argv)
{
    const std::string name = argc > 2 ? argv[2] : "gol_5.dc";
    dccrg::Dccrg<game_of_life_cell> ref, grid;
    for (auto* g : {&ref, &grid}) {
        g->set_initial_length({15, 15, 1}).set_neighborhood_length(1).set_maximum_refinement_level(-1)
            .initialize(MPI_COMM_WORLD);
        for (const auto& cell : g->local_cells()) cell.data->is_alive = splitmix64(cell.id) % 3 == 0;
    }
    for (int s = 0; s < 5; s++) gol_turn(grid);
    uint64_t step = 5;
    if (!grid.save_grid_data(name, 0, std::make_tuple((void*)&step, 1, MPI_UINT64_T))) abort();
    dccrg::Dccrg<game_of_life_cell> loaded;
    uint64_t read_step = 0;
    if (!loaded.load_grid_data(name, 0, std::make_tuple((void*)&read_step, 1, MPI_UINT64_T), MPI_COMM_WORLD, "RCB"))
        abort();
    if (read_step != 5) abort();
    if (loaded.get_maximum_refinement_level() != grid.get_maximum_refinement_level()) abort();
    for (int s = 0; s < 5; s++) gol_turn(loaded);
    for (int s = 0; s < 10; s++) gol_turn(ref);
    size_t n = 0;
    for (const auto& cell : ref.local_cells()) {
        if (!loaded[cell.id] || loaded[cell.id]->is_alive != cell.data->is_alive) abort();
        n++;
    }
    printf("PASS restart %zu\n", n);
    return 0;
}

static void print_lists(dccrg::Dccrg<uint64_t>& grid)
{
    for (const auto& cell : grid.local_cells()) {
        printf("cell %llu of", (unsigned long long)cell.id);
        for (const auto& n : cell.neighbors_of) printf(" %llu:%d,%d,%d", (unsigned long long)n.id, n.x, n.y, n.z);
        printf(" to");
        for (const auto& n : cell.neighbors_to) printf(" %llu:%d,%d,%d", (unsigned long long)n.id, n.x, n.y, n.z);
        printf("\n");
    }
}

static int amr(int argc, char** argv)
{
    dccrg::Dccrg<uint64_t> grid;
    grid.set_initial_length({6, 5, 4})
        .set_neighborhood_length(1)
        .set_maximum_refinement_level(1)
        .set_periodic(false, true, true)
        .initialize(MPI_COMM_WORLD);
    for (const auto& cell : grid.local_cells()) *cell.data = cell.id;
    std::vector<uint64_t> asked;
    for (int i = 2; i < argc; i++) {
        const uint64_t c = strtoull(argv[i], 0, 10);
        if (!grid.refine_completely(c)) abort();
        asked.push_back(c);
    }
    const auto created = grid.stop_refining(true);
    printf("new");
    for (uint64_t c : created) printf(" %llu", (unsigned long long)c);
    printf("\n");
    // refined parents keep their data until clear_refined_unrefined_data
    for (uint64_t c : asked)
        if (!grid[c] || *grid[c] != c) abort();
    for (uint64_t c : created) {
        if (!grid[c] || *grid[c] != 0) abort();  // value-initialised
        *grid[c] = *grid[grid.mapping.get_parent(c)];
    }
    grid.clear_refined_unrefined_data();
    for (uint64_t c : asked)
        if (grid[c]) abort();
    grid.update_copies_of_remote_neighbors();
    print_lists(grid);
    // unrefine back: the children's data stays readable, parents are new
    for (uint64_t c : created) grid.unrefine_completely(c);
    // execute_refines returns only the children of refined cells (dccrg.hpp:10374)
    if (!grid.stop_refining(true).empty()) abort();
    for (uint64_t c : asked)
        if (!grid.is_local(c) || *grid[c] != 0) abort();  // parents are new, value-initialised
    const auto removed = grid.get_removed_cells(true);
    if (removed.size() != created.size()) abort();
    for (uint64_t c : removed)
        if (!grid[c] || *grid[c] != grid.mapping.get_parent(c)) abort();
    printf("PASS amr\n");
    return 0;
}

static void print_matches(const char* tag, const std::vector<uint64_t>& ids)
{
    printf("%s", tag);
    for (uint64_t c : ids) printf(" %llu", (unsigned long long)c);
    printf("\n");
}

// get_cells(criteria, exact_match, hood) and the process-boundary accessors
// (dccrg.hpp:661, 2968, 6158-6300); a user neighborhood {+x} as hood 7
static int cells(int argc, char** argv)
{
    dccrg::Dccrg<int> grid;
    grid.set_initial_length({strtoull(argv[2], 0, 10), strtoull(argv[3], 0, 10), strtoull(argv[4], 0, 10)})
        .set_neighborhood_length(atoi(argv[8]))
        .set_maximum_refinement_level(0)
        .set_periodic(atoi(argv[5]), atoi(argv[6]), atoi(argv[7]))
        .initialize(MPI_COMM_WORLD);
    if (!grid.add_neighborhood(7, {{1, 0, 0}})) abort();
    const int crit[] = {dccrg::has_no_neighbor, dccrg::has_local_neighbor_of, dccrg::has_local_neighbor_to,
                        dccrg::has_local_neighbor_both, dccrg::has_remote_neighbor_of,
                        dccrg::has_remote_neighbor_both};
    for (int hood : {dccrg::default_neighborhood_id, 7}) {
        for (int c : crit)
            for (int exact : {0, 1}) {
                char tag[64];
                snprintf(tag, sizeof tag, "hood %d crit %d exact %d :", hood == 7 ? 7 : 0, c, exact);
                print_matches(tag, grid.get_cells({c}, exact, hood));
            }
        print_matches(hood == 7 ? "hood 7 all :" : "hood 0 all :", grid.get_cells({}, false, hood));
        if (!grid.get_local_cells_on_process_boundary(hood).empty()) abort();
        if (!grid.get_remote_cells_on_process_boundary(hood, true).empty()) abort();
        if (grid.get_local_cells_not_on_process_boundary(hood) != grid.get_cells()) abort();
    }
    if (!grid.get_cells({dccrg::has_local_neighbor_of}, false, 99).empty()) abort();  // unknown hood
    // the user-neighborhood views (dccrg.hpp:6860-6914, 6978-7044)
    if (grid.get_user_hood_of().at(7) != std::vector<std::array<int, 3>>{{{1, 0, 0}}}) abort();
    if (grid.get_user_hood_to().at(7) != std::vector<std::array<int, 3>>{{{-1, 0, 0}}}) abort();
    if (grid.get_user_hood_of().count(dccrg::default_neighborhood_id)) abort();
    if (!grid.get_user_local_cells_on_process_boundary().at(7).empty()) abort();  // one process
    if (!grid.get_user_remote_cells_on_process_boundary().at(7).empty()) abort();
    if (!grid.get_user_neigh_cells_to_send().at(7).empty() || !grid.get_user_neigh_cells_to_receive().at(7).empty())
        abort();
    for (uint64_t c : grid.get_cells()) {
        if (grid.get_all_neighbors_of().at(c) != *grid.get_neighbors_of(c)) abort();
        if (grid.get_all_neighbors_to().at(c) != *grid.get_neighbors_to(c)) abort();
    }
    for (uint64_t c : grid.get_cells()) {
        printf("face %llu :", (unsigned long long)c);
        for (const auto& f : grid.get_face_neighbors_of(c)) printf(" %llu/%d", (unsigned long long)f.first, f.second);
        printf("\n");
    }
    grid.allocate_copies_of_remote_neighbors(7);
    bool threw = false;
    try {
        grid.allocate_copies_of_remote_neighbors(99);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    if (!threw) abort();
    return 0;
}

// the coordinate lookups: get_existing_cell, refine_completely_at,
// dont_unrefine_at (dccrg.hpp:3401-3467, 6424-6444, 11414-11447) over the
// Cartesian geometry's get_indices / get_real_coordinate / get_cell
// (dccrg_cartesian_geometry.hpp:496-608), and get_remote_neighbors_to
// (dccrg.hpp:3225-3287) against the neighbor lists; aborts on a mismatch
static int coords()
{
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    dccrg::Dccrg<int, dccrg::Cartesian_Geometry> grid;
    grid.set_initial_length({4, 4, 2})
        .set_neighborhood_length(1)
        .set_maximum_refinement_level(2)
        .set_periodic(true, false, false)
        .initialize(MPI_COMM_WORLD);
    // x from -1 (4 cells of 0.5), y from 0 (4 of 1), z from 0 (2 of 2)
    grid.set_geometry(dccrg::Cartesian_Geometry::Parameters({{-1, 0, 0}}, {{0.5, 1, 2}}));
    auto want = [](bool ok, const char* what) {
        if (!ok) {
            std::fprintf(stderr, "FAIL %s\n", what);
            abort();
        }
    };
    const uint64_t err = dccrg::error_cell;
    want(grid.get_existing_cell({{-0.9, 0.1, 0.1}}) == 1, "first cell");
    want(grid.get_existing_cell({{0.9, 3.9, 3.9}}) == 32, "last cell");
    want(grid.get_existing_cell({{1.1, 0.1, 0.1}}) == 1, "periodic x wraps");
    want(grid.get_existing_cell({{-2.9, 0.1, 0.1}}) == 1, "periodic x wraps from below");
    want(grid.get_existing_cell({{0.0, -0.1, 0.1}}) == err, "outside non-periodic y");
    want(grid.get_existing_cell({{0.0, 4.0, 0.1}}) == err, "on the end face of y: index past the grid");
    want(grid.geometry.get_end()[0] == 1.0 && grid.geometry.get_end()[2] == 4.0, "get_end");
    const bool mine = grid.is_local(1);
    want(grid.refine_completely_at({{-0.9, 0.1, 0.1}}) == mine, "refine_completely_at on the owner");
    want(!grid.refine_completely_at({{0.0, 9.0, 0.0}}), "refine_completely_at outside");
    grid.stop_refining();
    const uint64_t child = grid.mapping.get_cell_from_indices({{0, 0, 0}}, 1);
    want(grid.get_existing_cell({{-0.9, 0.1, 0.1}}) == child, "smallest cell after refinement");
    want(grid.get_existing_cell({{0, 0, 0}}, 0, 0) == err, "level 0 only: the parent is gone");
    want(grid.get_existing_cell({{0, 0, 0}}, 0, 2) == child, "levels 0-2");
    want(grid.get_existing_cell({{0, 0, 0}}, 2, 1) == err, "min level > max level");
    want(grid.geometry.get_cell(1, {{-0.9, 0.1, 0.1}}) == child, "geometry get_cell");
    want(grid.geometry.get_cell(3, {{-0.9, 0.1, 0.1}}) == err, "geometry get_cell beyond the maximum level");
    const bool dont = grid.dont_unrefine_at({{-0.9, 0.1, 0.1}});
    if (grid.is_local(child)) want(dont, "dont_unrefine_at on the owner");
    want(!grid.dont_unrefine_at({{0.0, 9.0, 0.0}}), "dont_unrefine_at outside");
    const std::vector<uint64_t> all = grid.get_all_cells();
    want(all.size() == 31 + 8 && std::is_sorted(all.begin(), all.end()), "get_all_cells: 31 level-0 cells + 8");
    want(std::binary_search(all.begin(), all.end(), child) && !std::binary_search(all.begin(), all.end(), 1),
         "get_all_cells: the children, not the parent");
    const auto items = grid.get_neighborhood_of();
    want(items.size() == 26 && items.front() == (std::array<int, 3>{{-1, -1, -1}}) &&
             items.back() == (std::array<int, 3>{{1, 1, 1}}) &&
             grid.get_neighborhood_to().front() == (std::array<int, 3>{{1, 1, 1}}),
         "neighborhood items in z, y, x order");
    want(grid.get_max_tag() >= 32767u, "max tag");
    want(grid.get_cell_data().size() == grid.get_cells().size(), "cell data of the local cells");
    size_t n_remote = 0;
    for (uint64_t c : grid.get_cells()) {
        std::vector<uint64_t> of;
        for (const auto& x : *grid.get_neighbors_of(c))
            if (grid.get_process(x.first) != rank) of.push_back(x.first);
        std::sort(of.begin(), of.end());
        want(grid.get_remote_neighbors_of(c, dccrg::default_neighborhood_id, true) == of, "remote neighbors of");
        std::vector<uint64_t> brute;
        for (const auto& x : *grid.get_neighbors_to(c))
            if (grid.get_process(x.first) != rank) brute.push_back(x.first);
        std::sort(brute.begin(), brute.end());
        want(grid.get_remote_neighbors_to(c, dccrg::default_neighborhood_id, true) == brute, "remote neighbors to");
        n_remote += brute.size();
    }
    for (uint64_t c = 1; c <= 32; c++)
        if (!grid.is_local(c)) want(grid.get_remote_neighbors_to(c).empty(), "not local: nothing");
    want(grid.get_max_ref_lvl_diff() == 1 && grid.get_initialized() && grid.get_mapping_initialized(), "getters");
    // load balancing as built with DCCRG_NO_LB; cell weights (dccrg.hpp:5905-6130, 6318-6379)
    want(!grid.pin(child) && !grid.pin(child, 0) && !grid.unpin(child) && !grid.unpin_local_cells(), "no-LB pins");
    grid.unpin_all_cells();
    for (uint64_t c : grid.get_cells()) want(grid.get_cell_weight(c) == 1.0, "unset weight");
    want(std::isnan(grid.get_cell_weight(0)), "weight of a non-cell");
    if (grid.is_local(child)) {
        want(grid.set_cell_weight(child, 2.5) && grid.get_cell_weight(child) == 2.5, "set weight");
        want(grid.refine_completely(child), "refine the weighted cell");
    }
    grid.stop_refining();
    const uint64_t grandchild = grid.mapping.get_cell_from_indices({{0, 0, 0}}, 2);
    if (grid.is_local(grandchild)) {
        want(grid.get_cell_weight(grandchild) == 2.5, "children inherit the weight");
        want(grid.get_cell_weights().count(child) == 0, "the refined cell's weight is gone");
    }
    std::printf("coords ok rank %d remote_to %zu\n", rank, n_remote);
    return 0;
}

// tests/constructors/copy.cpp's cell types: the copy holds another type
struct copy_cell_1 {
    int data = -1;
    std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple((void*)&data, 1, MPI_INT); }
};
struct copy_cell_2 {
    double data = -2;
    std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple((void*)&data, 1, MPI_DOUBLE); }
};

// as copy.cpp checks them: the remote boundary set and the cell -> owner map
template <class G> static void check_remote_copies(const G& grid, double factor, const char* what)
{
    const std::unordered_set<uint64_t>& remote = grid.get_remote_cells_on_process_boundary_internal();
    const std::unordered_map<uint64_t, uint64_t>& cell_process = grid.get_cell_process();
    if (remote.size() != grid.get_remote_cells_on_process_boundary().size() ||
        cell_process.size() != grid.get_all_cells().size() ||
        grid.get_local_cells_on_process_boundary_internal().size() != grid.get_local_cells_on_process_boundary().size())
        abort();
    // the sets are kept between calls: a second call returns the same object
    if (&grid.get_cell_process() != &cell_process || &grid.get_remote_cells_on_process_boundary_internal() != &remote ||
        grid.get_cell_process().size() != cell_process.size())
        abort();
    for (uint64_t c : remote) {
        const auto* d = grid[c];
        if (d == nullptr || double(d->data) != factor * double(cell_process.at(c)) ||
            int(cell_process.at(c)) != grid.get_process(c)) {
            std::fprintf(stderr, "FAIL %s: cell %llu\n", what, (unsigned long long)c);
            abort();
        }
    }
}

// tests/constructors/copy.cpp, on a refined grid with a user neighborhood
// and a cell weight: the copy (another cell type, then another geometry)
// has the same cells, owners, lists and iterators, default-constructed
// data, and remote neighbor updates that work independently of the original
static int copy()
{
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    auto want = [](bool ok, const char* what) {
        if (!ok) {
            std::fprintf(stderr, "FAIL %s\n", what);
            abort();
        }
    };
    dccrg::Dccrg<copy_cell_1, dccrg::Cartesian_Geometry> grid1;
    grid1.set_initial_length({10, 10, 10})
        .set_neighborhood_length(1)
        .set_maximum_refinement_level(1)
        .set_periodic(true, false, false)
        .initialize(MPI_COMM_WORLD);
    grid1.set_geometry(dccrg::Cartesian_Geometry::Parameters({{-1, 0, 0}}, {{0.5, 1, 2}}));
    {
        bool threw = false;
        try {
            grid1.set_geometry(dccrg::Cartesian_Geometry::Parameters({{-1, 0, 0}}, {{-0.5, 1, 2}}));
        } catch (const std::invalid_argument&) {
            threw = true;
        }
        want(threw, "set_geometry rejects a negative cell length (dccrg.hpp:586-595 throws)");
    }
    if (grid1.is_local(456)) grid1.refine_completely(456);
    grid1.stop_refining();
    const std::vector<dccrg::Types<3>::neighborhood_item_t> items{{{0, 0, -1}}, {{0, 0, 1}}, {{1, 0, 0}}};
    want(grid1.add_neighborhood(7, items), "user neighborhood");
    const uint64_t child = grid1.get_all_cells().back();
    if (grid1.is_local(child)) want(grid1.set_cell_weight(child, 3.0), "weight");
    for (const auto& cell : grid1.local_cells()) cell.data->data = rank;
    grid1.update_copies_of_remote_neighbors();
    check_remote_copies(grid1, 1, "grid1 update");

    dccrg::Dccrg<copy_cell_2, dccrg::Cartesian_Geometry> grid2(grid1);
    want(grid2.get_initialized(), "initialized");
    want(grid2.get_all_cells() == grid1.get_all_cells() && grid2.get_cells() == grid1.get_cells(), "same cells");
    for (uint64_t c : grid1.get_all_cells()) want(grid2.get_process(c) == grid1.get_process(c), "same owners");
    want(grid2.geometry.get_start() == grid1.geometry.get_start() &&
             grid2.geometry.get_level_0_cell_length() == grid1.geometry.get_level_0_cell_length(),
         "geometry copied");
    want(grid2.get_neighborhood_length() == 1 && grid2.topology.is_periodic(0) && !grid2.topology.is_periodic(1) &&
             grid2.mapping.get_maximum_refinement_level() == 1,
         "parameters copied");
    want(grid2.get_user_hood_of() == grid1.get_user_hood_of() && grid2.get_cell_weights() == grid1.get_cell_weights(),
         "user neighborhoods and weights copied");
    for (uint64_t c : grid1.get_cells()) {
        want(*grid2.get_neighbors_of(c) == *grid1.get_neighbors_of(c), "neighbors_of");
        want(*grid2.get_neighbors_to(c) == *grid1.get_neighbors_to(c), "neighbors_to");
        want(*grid2.get_neighbors_of(c, 7) == *grid1.get_neighbors_of(c, 7), "user neighbors_of");
    }
    for (const auto& cell : grid2.local_cells()) want(cell.data->data == -2, "default-constructed data");
    want(size_t(std::distance(grid2.local_cells().begin(), grid2.local_cells().end())) == grid2.get_cells().size(),
         "local iterator");
    want(size_t(std::distance(grid2.inner_cells().begin(), grid2.inner_cells().end())) ==
             grid2.get_local_cells_not_on_process_boundary().size(),
         "inner iterator");
    want(size_t(std::distance(grid2.outer_cells().begin(), grid2.outer_cells().end())) ==
             grid2.get_local_cells_on_process_boundary().size(),
         "outer iterator");
    want(grid2.get_remote_cells_on_process_boundary() == grid1.get_remote_cells_on_process_boundary(),
         "remote cells on the process boundary");
    for (const auto& cell : grid2.local_cells()) cell.data->data = 2 * rank;
    grid2.update_copies_of_remote_neighbors();
    check_remote_copies(grid2, 2, "grid2 update");
    check_remote_copies(grid1, 1, "grid1 untouched");
    want(grid2.update_copies_of_remote_neighbors(7), "user neighborhood update");

    dccrg::Dccrg<copy_cell_1> grid3(grid2);  // and into another geometry
    want(grid3.get_all_cells() == grid1.get_all_cells() && grid3.get_cells() == grid1.get_cells(), "third grid");
    for (const auto& cell : grid3.local_cells()) want(cell.data->data == -1, "third grid data");
    std::printf("copy ok rank %d cells %zu\n", rank, grid2.get_cells().size());
    return 0;
}

// tests/variable_data_size/variable_neighbour_data.cpp's cell: two vectors,
// the first alone or both through a struct type of their addresses
static bool send_variables2 = false;
struct var_cell {
    std::vector<int> variables1, variables2;
    std::tuple<void*, int, MPI_Datatype> get_mpi_datatype()
    {
        if (!send_variables2) return std::make_tuple((void*)variables1.data(), int(variables1.size()), MPI_INT);
        int counts[2] = {int(variables1.size()), int(variables2.size())};
        MPI_Aint displacements[2] = {0, (uint8_t*)variables2.data() - (uint8_t*)variables1.data()};
        MPI_Datatype types[2] = {MPI_INT, MPI_INT}, t = MPI_DATATYPE_NULL;
        if (MPI_Type_create_struct(2, counts, displacements, types, &t) != MPI_SUCCESS)
            return std::make_tuple((void*)variables1.data(), 0, MPI_BYTE);
        return std::make_tuple((void*)variables1.data(), 1, t);
    }
};

// variable_neighbour_data.cpp:82-130 (its load-balancing half is out of
// scope): cell c holds c values c+i and -(c+i); receivers size the remote
// copies first; then the sizes change (2c) and only the first vector goes
static int varneigh(int argc, char** argv)
{
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    const uint64_t lx = argc > 2 ? strtoull(argv[2], 0, 10) : 3, ly = argc > 3 ? strtoull(argv[3], 0, 10) : 1;
    dccrg::Dccrg<var_cell> grid;
    grid.set_initial_length({lx, ly, 1}).set_neighborhood_length(1).set_maximum_refinement_level(0).initialize(
        MPI_COMM_WORLD);
    grid.allocate_copies_of_remote_neighbors();
    for (const auto& cell : grid.local_cells())
        for (uint64_t i = 0; i < cell.id; i++) {
            cell.data->variables1.push_back(int(cell.id + i));
            cell.data->variables2.push_back(-int(cell.id + i));
        }
    for (uint64_t c : grid.get_remote_cells_on_process_boundary()) {
        auto* d = grid[c];
        if (d == nullptr) abort();
        d->variables1.resize(c);
        d->variables2.resize(c);
    }
    send_variables2 = true;
    grid.update_copies_of_remote_neighbors();
    size_t checked = 0;
    for (const auto& cell : grid.local_cells())
        for (const auto& n : cell.neighbors_of) {
            if (n.data->variables1.size() != n.id || n.data->variables2.size() != n.id) abort();
            for (uint64_t i = 0; i < n.id; i++)
                if (n.data->variables1[i] != int(n.id + i) || n.data->variables2[i] != -int(n.id + i)) {
                    std::fprintf(stderr, "FAIL cell %llu neighbor %llu value %llu\n", (unsigned long long)cell.id,
                                 (unsigned long long)n.id, (unsigned long long)i);
                    abort();
                }
            checked++;
        }
    // new sizes; the first vector alone
    for (const auto& cell : grid.local_cells()) {
        cell.data->variables1.assign(2 * cell.id, 0);
        for (uint64_t i = 0; i < 2 * cell.id; i++) cell.data->variables1[i] = int(3 * cell.id + i);
    }
    for (uint64_t c : grid.get_remote_cells_on_process_boundary()) grid[c]->variables1.resize(2 * c);
    send_variables2 = false;
    grid.update_copies_of_remote_neighbors();
    for (const auto& cell : grid.local_cells())
        for (const auto& n : cell.neighbors_of) {
            if (n.data->variables1.size() != 2 * n.id) abort();
            for (uint64_t i = 0; i < 2 * n.id; i++)
                if (n.data->variables1[i] != int(3 * n.id + i)) abort();
            if (!grid.is_local(n.id) && n.data->variables2[0] != -int(n.id)) abort();  // untouched
        }
    std::printf("varneigh ok rank %d neighbors %zu\n", rank, checked);
    return 0;
}

// tests/user_neighborhood/game_of_life.cpp's known answer: the live cells of
// its four interlaced games (toad, blinker, beehive, beacon, block and a
// glider moving (2, -2) every 4 steps) on the 18 x 18 grid at a step that is
// a multiple of 4
static std::set<uint64_t> interlaced_live(int64_t gs, int step)
{
    std::set<uint64_t> r;
    const int64_t toad = 12 * gs + 6, blinker = 14 * gs + 1, hive = 10 * gs + 7, beacon = 15 * gs + 6,
                  block = 5 * gs + 2;
    for (int64_t v : {toad, toad + 2, toad + 4, toad + 2 + 2 * gs, toad + 4 + 2 * gs, toad + 6 + 2 * gs, blinker,
                      blinker + 2, blinker + 4, hive + 2, hive + 4, hive - 2 * gs, hive - 2 * gs + 6,
                      hive - 4 * gs + 2, hive - 4 * gs + 4, beacon, beacon + 2, beacon - 2 * gs, beacon + 6 - 4 * gs,
                      beacon + 4 - 6 * gs, beacon + 6 - 6 * gs, block, block + 2, block - 2 * gs, block + 2 - 2 * gs})
        r.insert(uint64_t(v));
    const int64_t k = step / 4;
    const int64_t glider[5][2] = {{3, 15}, {5, 13}, {1, 11}, {3, 11}, {5, 11}};
    for (const auto& g : glider) {
        const int64_t x = (g[0] + 2 * k) % gs, y = ((g[1] - 2 * k) % gs + gs) % gs;
        r.insert(uint64_t(y * gs + x));
    }
    return r;
}

// tests/user_neighborhood/game_of_life.cpp: a periodic 18 x 18 game over the
// user neighborhood {-2, 0, 2}^2 \ {0} (hood length 2), iterated with
// local_cells(hood) and updated with update_copies_of_remote_neighbors(hood);
// the live cells every 4 steps are the known answer above
static int interlaced()
{
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    const uint64_t gs = 18;
    dccrg::Dccrg<std::array<int, 2>> grid;
    grid.set_initial_length({gs, gs, 1})
        .set_neighborhood_length(2)
        .set_maximum_refinement_level(0)
        .set_periodic(true, true, true)
        .set_load_balancing_method("RANDOM")
        .initialize(MPI_COMM_WORLD);
    const std::vector<dccrg::Types<3>::neighborhood_item_t> hood{{{-2, -2, 0}}, {{-2, 0, 0}}, {{-2, 2, 0}},
                                                                 {{0, -2, 0}},  {{0, 2, 0}},  {{2, -2, 0}},
                                                                 {{2, 0, 0}},   {{2, 2, 0}}};
    const int hood_id = 1;
    if (!grid.add_neighborhood(hood_id, hood)) abort();
    for (uint64_t c : interlaced_live(gs, 0)) {
        auto* d = grid[c];
        if (d != nullptr) (*d)[0] = 1;
    }
    size_t checked = 0;
    for (int step = 0; step < 36; step++) {
        grid.balance_load();
        grid.update_copies_of_remote_neighbors(hood_id);
        if (step % 4 == 0) {
            const auto live = interlaced_live(gs, step);
            for (const auto& cell : grid.local_cells(hood_id)) {
                if (((*cell.data)[0] != 0) != (live.count(cell.id) > 0)) {
                    std::fprintf(stderr, "FAIL cell %llu step %d alive %d\n", (unsigned long long)cell.id, step,
                                 (*cell.data)[0]);
                    abort();
                }
                checked++;
            }
        }
        for (const auto& cell : grid.local_cells(hood_id)) {
            (*cell.data)[1] = 0;
            for (const auto& n : cell.neighbors_of)
                if ((*n.data)[0] == 1) (*cell.data)[1]++;
        }
        for (const auto& cell : grid.local_cells(hood_id)) {
            if ((*cell.data)[1] == 3) (*cell.data)[0] = 1;
            else if ((*cell.data)[1] != 2) (*cell.data)[0] = 0;
        }
    }
    std::printf("interlaced ok rank %d checked %zu\n", rank, checked);
    return 0;
}

// tests/additional_cell_data/{test1,test2,neighbor_data1,neighbor_data2}.cpp:
// a cell with no data, additional cell / neighbor items with defaults or
// filled in by update() (ids, No_Geometry centers), seen through grid.cells,
// local_cells() and neighbors_of, again after balance_load
struct empty_cell {
    std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple((void*)this, 0, MPI_BYTE); }
};
struct aci_defaults_1 {
    int additional_cell_data1 = 1;
    double additional_cell_data2 = 3.125;
    template <class Grid, class Cell> void update(const Grid&, const Cell&, const aci_defaults_1&) {}
};
struct aci_defaults_2 {
    std::tuple<int, float> additional_cell_data3{2, 3.0625f};
    unsigned int additional_cell_data4 = 4;
    template <class Grid, class Cell> void update(const Grid&, const Cell&, const aci_defaults_2&) {}
};
struct aci_id {
    uint64_t additional_cell_data1 = dccrg::error_cell;
    template <class Grid, class Cell> void update(const Grid&, const Cell& cell, const aci_id&)
    {
        additional_cell_data1 = cell.id;
    }
};
struct aci_center {
    double d1 = 0, d2 = 0, d3 = 0;
    uint64_t additional_cell_data4 = dccrg::error_cell;
    template <class Grid, class Cell> void update(const Grid& grid, const Cell& cell, const aci_center&)
    {
        additional_cell_data4 = cell.id;
        const auto c = grid.geometry.get_center(cell.id);
        d1 = c[0];
        d2 = c[1];
        d3 = c[2];
    }
};
struct ani_defaults {
    int additional_neighbor_data1 = 1;
    double additional_neighbor_data2 = 3.125;
    template <class Grid, class C, class N> void update(const Grid&, const C&, const N&, const int&, const ani_defaults&)
    {
    }
};
struct ani_ids {
    uint64_t additional_neighbor_data1 = dccrg::error_cell, additional_neighbor_data2 = dccrg::error_cell;
    template <class Grid, class C, class N>
    void update(const Grid&, const C& cell, const N& neighbor, const int&, const ani_ids&)
    {
        additional_neighbor_data1 = neighbor.id;
        additional_neighbor_data2 = cell.id;
    }
};

template <class G> static void setup_items_grid(G& grid)
{
    grid.set_initial_length({2, 2, 2})
        .set_neighborhood_length(3)
        .set_maximum_refinement_level(-1)
        .set_load_balancing_method("RANDOM")
        .initialize(MPI_COMM_WORLD);
}

static int items()
{
    int rank = 0, size = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    auto want = [](bool ok, const char* what) {
        if (!ok) {
            std::fprintf(stderr, "FAIL %s\n", what);
            abort();
        }
    };
    {  // test1.cpp
        dccrg::Dccrg<empty_cell, dccrg::No_Geometry, std::tuple<aci_defaults_1, aci_defaults_2>> grid;
        setup_items_grid(grid);
        want(grid.cells.size() == size_t(std::distance(grid.all_cells().begin(), grid.all_cells().end())) &&
                 grid.cells.size() >= grid.get_cells().size(),
             "cells: local and remote copies");
        for (const auto& cell : grid.cells)
            want(cell.additional_cell_data1 == 1 && cell.additional_cell_data2 == 3.125 &&
                     std::get<0>(cell.additional_cell_data3) == 2 &&
                     std::get<1>(cell.additional_cell_data3) == 3.0625f && cell.additional_cell_data4 == 4,
                 "default cell items");
        // No_Geometry (dccrg_no_geometry.hpp): unit level-0 cells from the origin
        const int top = grid.mapping.get_maximum_refinement_level();
        want(top == grid.mapping.get_maximum_possible_refinement_level(), "maximum level -1: the largest possible");
        const auto& g = grid.geometry;
        want(g.get_end() == (std::array<double, 3>{{2, 2, 2}}) && g.get_start() == (std::array<double, 3>{{0, 0, 0}}),
             "no geometry corners");
        want(g.get_center(8) == (std::array<double, 3>{{1.5, 1.5, 1.5}}) &&
                 g.get_length(8) == (std::array<double, 3>{{1, 1, 1}}) &&
                 g.get_min(2) == (std::array<double, 3>{{1, 0, 0}}),
             "no geometry level-0 cells");
        const uint64_t child = grid.mapping.get_cell_from_indices({{0, 0, 0}}, 1);
        want(g.get_center(child) == (std::array<double, 3>{{0.25, 0.25, 0.25}}) &&
                 g.get_max(child) == (std::array<double, 3>{{0.5, 0.5, 0.5}}),
             "no geometry level-1 cell");
        want(std::isnan(g.get_center(dccrg::error_cell)[0]) && std::isnan(g.get_length(0)[1]), "no geometry errors");
        want(std::isnan(g.get_real_coordinate({{-0.5, 1, 1}})[0]) && g.get_real_coordinate({{-0.5, 1, 1}})[1] == 1,
             "no geometry outside a non-periodic dimension");
        want(g.get_indices({{1.5, 0.25, 2.0}}) == (dccrg::Types<3>::indices_t{{1, 0, 2}}) &&
                 g.get_indices({{2.5, 0, 0}})[0] == dccrg::error_index,
             "no geometry indices (the floor of the coordinate)");
        want(g.get_cell(0, {{0.5, 0.5, 0.5}}) == 1 && g.get_cell(top + 1, {{0.5, 0.5, 0.5}}) == dccrg::error_cell,
             "no geometry get_cell");
        const auto cc = g.get_center(0, {{uint64_t(1) << top, 0, 0}});
        want(cc[0] == 1.5 && cc[1] == 0.5 && std::isnan(g.get_center(0, {{uint64_t(3) << top, 0, 0}})[0]),
             "no geometry center at indices");
    }
    {  // test2.cpp
        dccrg::Dccrg<empty_cell, dccrg::No_Geometry, std::tuple<aci_id, aci_center>> grid;
        setup_items_grid(grid);
        auto check = [&](const char* what) {
            for (const auto& cell : grid.cells) {
                const auto c = grid.geometry.get_center(cell.id);
                want(cell.additional_cell_data1 == cell.id && cell.additional_cell_data4 == cell.id &&
                         cell.d1 == c[0] && cell.d2 == c[1] && cell.d3 == c[2],
                     what);
            }
        };
        check("updated cell items");
        for (auto& cell : grid.cells) {
            const_cast<uint64_t&>(cell.additional_cell_data1) = dccrg::error_cell;
            const_cast<uint64_t&>(cell.additional_cell_data4) = dccrg::error_cell;
            const_cast<double&>(cell.d1) -= 3;
        }
        grid.balance_load();  // DCCRG_NO_LB: a no-op, the items keep what was written
        for (const auto& cell : grid.cells)
            want(cell.additional_cell_data1 == dccrg::error_cell, "balance_load left the cell items alone");
        grid.refresh_additional_items();
        check("cell items updated again by refresh_additional_items");
    }
    {  // neighbor_data1.cpp
        dccrg::Dccrg<empty_cell, dccrg::No_Geometry, std::tuple<>, std::tuple<ani_defaults>> grid;
        setup_items_grid(grid);
        size_t n = 0;
        for (const auto& cell : grid.local_cells())
            for (const auto& neighbor : cell.neighbors_of) {
                want(neighbor.additional_neighbor_data1 == 1 && neighbor.additional_neighbor_data2 == 3.125,
                     "default neighbor items");
                n++;
            }
        want(n == 7 * grid.get_cells().size(), "every other cell is a neighbor (hood 3 on 2x2x2)");
    }
    {  // neighbor_data2.cpp
        dccrg::Dccrg<empty_cell, dccrg::No_Geometry, std::tuple<>, std::tuple<ani_ids>> grid;
        setup_items_grid(grid);
        for (int round = 0; round < 2; round++) {
            for (const auto& cell : grid.local_cells())
                for (const auto& neighbor : cell.neighbors_of)
                    want(neighbor.additional_neighbor_data1 == neighbor.id &&
                             neighbor.additional_neighbor_data2 == cell.id,
                         "updated neighbor items");
            grid.balance_load();
        }
        grid.update_copies_of_remote_neighbors();  // zero-byte cells
    }
    std::printf("items ok rank %d of %d\n", rank, size);
    return 0;
}

// tests/constructors/simple.cpp: cell data is constructed in place, never
// copied, moved or assigned (each of those throws here), through
// initialization, remote copies, halo updates and rebuilt caches
struct no_copy_cell {
    double data = 0;
    no_copy_cell() = default;
    no_copy_cell(const no_copy_cell&) { throw std::runtime_error("cell copied"); }
    no_copy_cell(no_copy_cell&&) { throw std::runtime_error("cell moved"); }
    no_copy_cell& operator=(const no_copy_cell&) { throw std::runtime_error("cell assigned"); }
    no_copy_cell& operator=(no_copy_cell&&) { throw std::runtime_error("cell move-assigned"); }
    std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple((void*)&data, 1, MPI_DOUBLE); }
};

static int nocopy()
{
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    {
        dccrg::Dccrg<no_copy_cell> grid;
        grid.set_initial_length({1, 1, 1}).set_neighborhood_length(1).set_maximum_refinement_level(0).initialize(
            MPI_COMM_WORLD);
        for (const auto& cell : grid.local_cells()) cell.data->data = 1;
    }
    dccrg::Dccrg<no_copy_cell> grid;
    grid.set_initial_length({6, 4, 1}).set_neighborhood_length(1).set_maximum_refinement_level(1).initialize(
        MPI_COMM_WORLD);
    for (const auto& cell : grid.local_cells()) cell.data->data = double(cell.id);
    grid.update_copies_of_remote_neighbors();
    grid.balance_load();
    for (const auto& cell : grid.local_cells())
        for (const auto& n : cell.neighbors_of)
            if (n.data->data != double(n.id)) abort();
    grid.update_copies_of_remote_neighbors();  // refinement moves data aside (the reference copies it)
    std::printf("nocopy ok rank %d cells %zu\n", rank, grid.get_cells().size());
    return 0;
}

// dccrg.hpp:3320-3390's write_vtk_file after refinement and the no-LB
// three-phase balance_load; prints each local leaf's corners for the check
static int vtk(int argc, char** argv)
{
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    dccrg::Dccrg<int, dccrg::Cartesian_Geometry> grid;
    grid.set_initial_length({3, 2, 1}).set_neighborhood_length(1).set_maximum_refinement_level(1).initialize(
        MPI_COMM_WORLD);
    grid.set_geometry(dccrg::Cartesian_Geometry::Parameters({{-1, 0, 0}}, {{0.5, 1, 2}}));
    if (grid.is_local(2)) grid.refine_completely(2);
    grid.stop_refining();
    grid.initialize_balance_load(true);
    if (!grid.get_cells_added_by_balance_load().empty() || !grid.get_cells_removed_by_balance_load().empty()) abort();
    grid.continue_balance_load();
    grid.finish_balance_load();
    const std::string name = std::string(argc > 2 ? argv[2] : "grid") + "_" + std::to_string(rank) + ".vtk";
    if (!grid.write_vtk_file(name)) abort();
    for (uint64_t c : grid.get_cells()) {
        const auto lo = grid.geometry.get_min(c), hi = grid.geometry.get_max(c);
        std::printf("leaf %d %llu %.17g %.17g %.17g %.17g %.17g %.17g\n", rank, (unsigned long long)c, lo[0], lo[1],
                    lo[2], hi[0], hi[1], hi[2]);
    }
    return 0;
}

static void live_neighbor_counts(const dccrg::Dccrg<game_of_life_cell>::Iterator_Storage<
                                     dccrg::Dccrg<game_of_life_cell>::Cells_Item>& cells)
{
    for (const auto& cell : cells) {
        cell.data->live_neighbor_count = 0;
        for (const auto& neighbor : cell.neighbors_of)
            if (neighbor.data->is_alive) cell.data->live_neighbor_count++;
    }
}

static void apply_rules(const dccrg::Dccrg<game_of_life_cell>::Iterator_Storage<
                        dccrg::Dccrg<game_of_life_cell>::Cells_Item>& cells)
{
    for (const auto& cell : cells) {
        if (cell.data->live_neighbor_count == 3) cell.data->is_alive = 1;
        else if (cell.data->live_neighbor_count != 2) cell.data->is_alive = 0;
    }
}

static int overlap(int argc, char** argv)
{
    if (argc < 9) abort();
    dccrg::Dccrg<game_of_life_cell> grid;
    grid.set_initial_length({{strtoull(argv[2], 0, 10), strtoull(argv[3], 0, 10), strtoull(argv[4], 0, 10)}})
        .set_neighborhood_length(1)
        .set_maximum_refinement_level(0)
        .set_periodic(atoi(argv[6]) != 0, atoi(argv[7]) != 0, atoi(argv[8]) != 0)
        .initialize(MPI_COMM_WORLD)
        .balance_load();
    grid.set_send_single_cells(true);
    if (!grid.get_send_single_cells()) abort();
    const int turns = atoi(argv[5]);
    const auto &local_cells = grid.local_cells(), &inner_cells = grid.inner_cells(),
               &outer_cells = grid.outer_cells();
    for (const auto& cell : local_cells) {
        cell.data->live_neighbor_count = 0;
        cell.data->is_alive = splitmix64(cell.id) % 1000 < 200;
    }
    // get_neighbors_of_at_offset (dccrg.hpp:3100-3161): on a level-0 grid the
    // neighbor at each default item's offset is found there
    for (const auto& cell : local_cells) {
        const auto* nof = grid.get_neighbors_of(cell.id);
        for (const auto& n : *nof) {
            const auto at = grid.get_neighbors_of_at_offset(cell.id, n.second[0], n.second[1], n.second[2]);
            if (std::find(at.begin(), at.end(), n) == at.end()) abort();
        }
        if (!grid.get_neighbors_of_at_offset(cell.id, 0, 0, 0).empty()) abort();
    }
    for (int turn = 0; turn < turns; turn++) {
        grid.start_remote_neighbor_copy_receives();
        grid.start_remote_neighbor_copy_sends();
        live_neighbor_counts(inner_cells);
        grid.wait_remote_neighbor_copy_update_receives();
        live_neighbor_counts(outer_cells);
        apply_rules(inner_cells);
        grid.wait_remote_neighbor_copy_update_sends();
        apply_rules(outer_cells);
    }
    for (const auto& cell : local_cells)
        if (cell.data->is_alive)
            printf("alive %llu %u\n", (unsigned long long)cell.id, cell.data->live_neighbor_count);
    return 0;
}

int main(int argc, char** argv)
{
    if (MPI_Init(&argc, &argv) != MPI_SUCCESS) abort();
    int rc = 1;
    {
        const std::string mode = argc > 1 ? argv[1] : "blinker";
        if (mode == "blinker") rc = blinker();
        else if (mode == "scal3d") rc = scal3d(argc, argv);
        else if (mode == "halo") rc = halo();
        else if (mode == "mapping") rc = mapping();
        else if (mode == "lists") rc = lists(argc, argv);
        else if (mode == "amr") rc = amr(argc, argv);
        else if (mode == "restart") rc = restart(argc, argv);
        else if (mode == "cells") rc = cells(argc, argv);
        else if (mode == "overlap") rc = overlap(argc, argv);
        else if (mode == "coords") rc = coords();
        else if (mode == "copy") rc = copy();
        else if (mode == "varneigh") rc = varneigh(argc, argv);
        else if (mode == "interlaced") rc = interlaced();
        else if (mode == "items") rc = items();
        else if (mode == "nocopy") rc = nocopy();
        else if (mode == "vtk") rc = vtk(argc, argv);
    }
    MPI_Finalize();
    return rc;
}
