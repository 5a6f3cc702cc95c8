/* TEST INFRASTRUCTURE ONLY.  A driver of the REFERENCE's own Mapping,
 * Grid_Topology and Cartesian_Geometry classes, compiled from the headers
 * where they lie under /root/reference (oracle/Makefile target _ref/, output
 * only into oracle/_ref/).  These three headers need nothing but the C++
 * standard library and mpi.h (MPICH in /opt/conda), so unlike dccrg.hpp
 * (Boost.TTI, Zoltan) they build here without stand-ins.  The program is run
 * only by tests/golden/make_ref_mapping.py in the container that has the
 * reference, to write tests/golden/ref_mapping.npz; the tests compare the
 * oracle restatement and the device kernels with those vectors.
 *
 * Functions exercised (dccrg_mapping.hpp / dccrg_cartesian_geometry.hpp):
 *   get_indices :218-254, get_refinement_level :262-290,
 *   get_cell_length_in_indices :298-311, get_maximum_possible_refinement_level
 *   :317-330, get_child :339-360, get_parent :368-384, get_all_children
 *   :392-442, get_siblings :450-471, get_level_0_parent :480-494,
 *   get_last_cell :500-503, get_cell_from_indices :154-209;
 *   Cartesian_Geometry get_length :284-309, get_center :318-364,
 *   get_min :378-400, get_max :404-422.
 *
 * argv: Lx Ly Lz max_ref_lvl(<0: maximum possible, as Dccrg::
 *       set_maximum_refinement_level :8276) sx sy sz l0x l0y l0z
 * stdin (little endian): u64 n, n x u64 id, u64 m, m x (3 x u64 index, i64 level)
 * stdout: i64 max_ref_lvl, u64 last_cell, i64 max_possible,
 *         n records of 28 u64 + 12 f64, then m x u64 cell.
 */
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dccrg_cartesian_geometry.hpp"
#include "dccrg_length.hpp"
#include "dccrg_mapping.hpp"
#include "dccrg_topology.hpp"

static void get(void* p, size_t bytes)
{
    if (fread(p, 1, bytes, stdin) != bytes) {
        fprintf(stderr, "ref_mapping: short input\n");
        exit(2);
    }
}

static void put(const void* p, size_t bytes)
{
    if (fwrite(p, 1, bytes, stdout) != bytes) exit(3);
}

int main(int argc, char** argv)
{
    if (argc != 11) {
        fprintf(stderr, "usage: %s Lx Ly Lz max_ref_lvl sx sy sz l0x l0y l0z\n", argv[0]);
        return 1;
    }
    const std::array<uint64_t, 3> length{{strtoull(argv[1], nullptr, 10), strtoull(argv[2], nullptr, 10),
                                          strtoull(argv[3], nullptr, 10)}};
    int lvl = atoi(argv[4]);
    const std::array<double, 3> start{{atof(argv[5]), atof(argv[6]), atof(argv[7])}};
    const std::array<double, 3> l0{{atof(argv[8]), atof(argv[9]), atof(argv[10])}};

    dccrg::Grid_Length grid_length(length);
    dccrg::Mapping mapping(length);
    const int max_possible = mapping.get_maximum_possible_refinement_level();
    if (lvl < 0) lvl = max_possible;
    if (!mapping.set_maximum_refinement_level(lvl)) {
        fprintf(stderr, "ref_mapping: level %d not possible\n", lvl);
        return 1;
    }
    dccrg::Grid_Topology topology;
    dccrg::Cartesian_Geometry geometry(grid_length, mapping, topology);
    if (!geometry.set(dccrg::Cartesian_Geometry_Parameters(start, l0))) {
        fprintf(stderr, "ref_mapping: geometry rejected\n");
        return 1;
    }

    const int64_t hdr[3] = {lvl, (int64_t)mapping.get_last_cell(), max_possible};
    put(hdr, sizeof hdr);

    uint64_t n = 0;
    get(&n, 8);
    std::vector<uint64_t> ids(n);
    if (n) get(ids.data(), 8 * n);
    for (const uint64_t id : ids) {
        uint64_t r[28];
        const auto idx = mapping.get_indices(id);
        const int level = mapping.get_refinement_level(id);
        r[0] = idx[0];
        r[1] = idx[1];
        r[2] = idx[2];
        r[3] = (uint64_t)(int64_t)level;
        r[4] = mapping.get_cell_length_in_indices(id);
        r[5] = mapping.get_parent(id);
        r[6] = mapping.get_level_0_parent(id);
        r[7] = mapping.get_child(id);
        const auto ch = mapping.get_all_children(id);
        const auto sb = mapping.get_siblings(id);
        for (int i = 0; i < 8; i++) {
            r[8 + i] = ch[i];
            r[16 + i] = sb[i];
        }
        r[24] = mapping.get_cell_from_indices(idx, level);
        r[25] = r[26] = r[27] = 0;
        put(r, sizeof r);
        double g[12];
        const auto len = geometry.get_length(id), cen = geometry.get_center(id), mn = geometry.get_min(id),
                   mx = geometry.get_max(id);
        for (int k = 0; k < 3; k++) {
            g[k] = len[k];
            g[3 + k] = cen[k];
            g[6 + k] = mn[k];
            g[9 + k] = mx[k];
        }
        put(g, sizeof g);
    }

    uint64_t m = 0;
    get(&m, 8);
    for (uint64_t i = 0; i < m; i++) {
        uint64_t in[4];
        get(in, sizeof in);
        const dccrg::Types<3>::indices_t idx{{in[0], in[1], in[2]}};
        const uint64_t cell = mapping.get_cell_from_indices(idx, (int)(int64_t)in[3]);
        put(&cell, 8);
    }
    return 0;
}
