/*
 * dccrg_amd.hpp -- C++ drop-in facade of dccrg::Dccrg / dccrg::Mapping for the
 * hot path, implemented over the C-ABI of libdccrgx.so (include/dccrgx.h).
 *
 * Kept from the reference interface (dccrg.hpp:151-7186, dccrg_mapping.hpp):
 * chained setters, initialize(MPI_Comm), local/inner/outer/remote/all_cells()
 * with Cells_Item{id, data, neighbors_of, neighbors_to, all_neighbors} and
 * Neighbors_Item{id, data, x, y, z}, operator[], get_neighbors_of/_to,
 * add/remove_neighborhood, the per-peer send/receive lists and the halo
 * calls (update_copies_of_remote_neighbors, start_/wait_...), and Mapping's
 * id <-> index functions.  Cell data of arbitrary Cell_Data types stays on
 * the host as in the reference (pointers from operator[] are stable); its
 * halo bytes are produced with MPI_Pack from get_mpi_datatype() exactly as
 * the reference's struct datatypes describe them and moved per peer with
 * RCCL.  Neighbor lists, classification and send/receive lists are built on
 * the GPU.  The device-speed path (SoA fields + device stencils) is the C-ABI
 * itself (dccrgx_field_*, dccrgx_gol_*), reachable via device_grid().
 *
 * Adaptive refinement: refine_completely / unrefine_completely /
 * dont_refine / dont_unrefine record this rank's requests in libdccrgx;
 * stop_refining() all-gathers the four request sets with MPI_Allgatherv and
 * hands their union to dccrgx_stop_refining, which makes the reference's
 * decisions (override / induce / execute, dccrg.hpp:9730-10693) and rebuilds
 * the device structures; the facade then moves host cell data exactly as the
 * reference does (refined parents and removed children stay readable through
 * operator[] until clear_refined_unrefined_data, new cells are
 * value-initialised) and rebuilds its iteration caches.
 *
 * MPI is used for bootstrap (rank, size, broadcasting the RCCL id) and for
 * the all-gather of refinement requests.  Load balancing (Zoltan) is not part
 * of this path: balance_load() keeps the reference's non-Zoltan block
 * partition.
 */
#ifndef DCCRG_AMD_HPP
#define DCCRG_AMD_HPP

#include <mpi.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <limits>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <iterator>
#include <fstream>
#include <iostream>
#include <sstream>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "dccrgx.h"

namespace dccrg {

static const uint64_t error_cell = DCCRGX_ERROR_CELL;    // dccrg_mapping.hpp:38
static const uint64_t error_index = DCCRGX_ERROR_INDEX;  // dccrg_mapping.hpp:41
static const int default_neighborhood_id = DCCRGX_DEFAULT_NEIGHBORHOOD_ID;  // dccrg.hpp:99
// neighbor-type criteria of get_cells (dccrg.hpp:103-114)
static const int has_no_neighbor = 0;
static const int has_local_neighbor_of = 1 << 0;
static const int has_local_neighbor_to = 1 << 1;
static const int has_remote_neighbor_of = 1 << 2;
static const int has_remote_neighbor_to = 1 << 3;
static const int has_local_neighbor_both = has_local_neighbor_of | has_local_neighbor_to;
static const int has_remote_neighbor_both = has_remote_neighbor_of | has_remote_neighbor_to;

template <unsigned N> struct Types;
template <> struct Types<3> {  // dccrg_types.hpp:34-86
    typedef std::array<uint64_t, 3> indices_t;
    typedef std::array<int, 3> neighborhood_item_t;
};

namespace detail {

inline void check(int status, const char* what)
{
    if (status != DCCRGX_OK) throw std::runtime_error(std::string(what) + ": " + dccrgx_last_error());
}

// MPI datatype of builtin cell data (dccrg_get_cell_datatype.hpp:226-281)
template <class T> inline MPI_Datatype builtin_type();
template <> inline MPI_Datatype builtin_type<char>() { return MPI_CHAR; }
template <> inline MPI_Datatype builtin_type<signed char>() { return MPI_SIGNED_CHAR; }
template <> inline MPI_Datatype builtin_type<unsigned char>() { return MPI_UNSIGNED_CHAR; }
template <> inline MPI_Datatype builtin_type<short>() { return MPI_SHORT; }
template <> inline MPI_Datatype builtin_type<unsigned short>() { return MPI_UNSIGNED_SHORT; }
template <> inline MPI_Datatype builtin_type<int>() { return MPI_INT; }
template <> inline MPI_Datatype builtin_type<unsigned>() { return MPI_UNSIGNED; }
template <> inline MPI_Datatype builtin_type<long>() { return MPI_LONG; }
template <> inline MPI_Datatype builtin_type<unsigned long>() { return MPI_UNSIGNED_LONG; }
template <> inline MPI_Datatype builtin_type<long long>() { return MPI_LONG_LONG; }
template <> inline MPI_Datatype builtin_type<unsigned long long>() { return MPI_UNSIGNED_LONG_LONG; }
template <> inline MPI_Datatype builtin_type<float>() { return MPI_FLOAT; }
template <> inline MPI_Datatype builtin_type<double>() { return MPI_DOUBLE; }
template <> inline MPI_Datatype builtin_type<long double>() { return MPI_LONG_DOUBLE; }

template <class C, class = void> struct has_gmd5 : std::false_type {};
template <class C>
struct has_gmd5<C, decltype(void(std::declval<C&>().get_mpi_datatype(uint64_t(), int(), int(), bool(), int())))>
    : std::true_type {};
template <class C, class = void> struct has_gmd0 : std::false_type {};
template <class C>
struct has_gmd0<C, decltype(void(std::declval<C&>().get_mpi_datatype()))> : std::true_type {};
template <class T> struct is_std_array : std::false_type {};
template <class T, size_t N> struct is_std_array<std::array<T, N>> : std::true_type {};

// the (address, count, datatype) a cell puts on the wire, dccrg_get_cell_datatype.hpp:48-339:
// get_mpi_datatype(id, sender, receiver, receiving, hood), get_mpi_datatype(),
// a builtin, or a std::array of builtins -- chosen in that order (tag dispatch)
template <class C>
struct datatype_kind
    : std::integral_constant<int, has_gmd5<C>::value ? 0 : has_gmd0<C>::value ? 1 : std::is_arithmetic<C>::value ? 2 : 3> {
};
template <class C>
std::tuple<void*, int, MPI_Datatype> cell_datatype_(C& c, uint64_t id, int s, int r, bool rc, int h,
                                                    std::integral_constant<int, 0>)
{
    return c.get_mpi_datatype(id, s, r, rc, h);
}
template <class C>
std::tuple<void*, int, MPI_Datatype> cell_datatype_(C& c, uint64_t, int, int, bool, int, std::integral_constant<int, 1>)
{
    return c.get_mpi_datatype();
}
template <class C>
std::tuple<void*, int, MPI_Datatype> cell_datatype_(C& c, uint64_t, int, int, bool, int, std::integral_constant<int, 2>)
{
    return std::make_tuple((void*)&c, 1, builtin_type<C>());
}
template <class C>
std::tuple<void*, int, MPI_Datatype> cell_datatype_(C& c, uint64_t, int, int, bool, int, std::integral_constant<int, 3>)
{
    static_assert(is_std_array<C>::value, "Cell_Data needs get_mpi_datatype() or must be a builtin / std::array");
    return std::make_tuple((void*)c.data(), (int)c.size(), builtin_type<typename C::value_type>());
}
template <class C>
std::tuple<void*, int, MPI_Datatype> cell_datatype(C& c, uint64_t id, int sender, int receiver, bool receiving,
                                                   int hood)
{
    return cell_datatype_(c, id, sender, receiver, receiving, hood, datatype_kind<C>());
}

// dccrg_mpi_support.hpp:66-95
inline bool is_named(MPI_Datatype t)
{
    int ni = 0, na = 0, nd = 0, comb = 0;
    MPI_Type_get_envelope(t, &ni, &na, &nd, &comb);
    return comb == MPI_COMBINER_NAMED;
}

// A derived datatype as byte blocks (displacement from the cell's address,
// length) in type-map order.  On a homogeneous run MPI_Pack's bytes are these
// blocks concatenated, so a cell is packed by memcpy instead of
// MPI_Type_commit + MPI_Pack + MPI_Type_free per cell and exchange (the
// reference commits every cell's type per exchange, dccrg.hpp:10850-10925).
// Combiners outside the usual constructors (subarray, darray, Fortran types)
// return false and are packed through MPI.
struct Blocks {
    std::vector<std::pair<MPI_Aint, MPI_Aint>> b;
    MPI_Aint bytes = 0;
    void add(MPI_Aint d, MPI_Aint n)
    {
        if (n <= 0) return;
        bytes += n;
        if (!b.empty() && b.back().first + b.back().second == d) b.back().second += n;
        else b.emplace_back(d, n);
    }
};

inline bool flatten(MPI_Datatype t, MPI_Aint count, MPI_Aint disp, Blocks& out, int depth = 0)
{
    if (depth > 32) return false;
    int ni = 0, na = 0, nd = 0, comb = 0;
    MPI_Type_get_envelope(t, &ni, &na, &nd, &comb);
    MPI_Aint lb = 0, ext = 0;
    MPI_Type_get_extent(t, &lb, &ext);
    if (comb == MPI_COMBINER_NAMED) {
        int sz = 0;
        MPI_Type_size(t, &sz);
        if ((MPI_Aint)sz == ext) out.add(disp, count * sz);  // contiguous repetitions
        else
            for (MPI_Aint c = 0; c < count; c++) out.add(disp + c * ext, sz);  // e.g. MPI_DOUBLE_INT's gap
        return true;
    }
    std::vector<int> ints(ni);
    std::vector<MPI_Aint> adds(na);
    std::vector<MPI_Datatype> types(nd);
    MPI_Type_get_contents(t, ni, na, nd, ints.data(), adds.data(), types.data());
    MPI_Aint lb0 = 0, ext0 = 0;
    if (nd) MPI_Type_get_extent(types[0], &lb0, &ext0);
    bool ok = true;
    for (MPI_Aint c = 0; c < count && ok; c++) {
        const MPI_Aint at = disp + c * ext;
        switch (comb) {
        case MPI_COMBINER_DUP:
        case MPI_COMBINER_RESIZED: ok = flatten(types[0], 1, at, out, depth + 1); break;
        case MPI_COMBINER_CONTIGUOUS: ok = flatten(types[0], ints[0], at, out, depth + 1); break;
        case MPI_COMBINER_VECTOR:
            for (int i = 0; i < ints[0] && ok; i++)
                ok = flatten(types[0], ints[1], at + (MPI_Aint)i * ints[2] * ext0, out, depth + 1);
            break;
        case MPI_COMBINER_HVECTOR:
            for (int i = 0; i < ints[0] && ok; i++) ok = flatten(types[0], ints[1], at + i * adds[0], out, depth + 1);
            break;
        case MPI_COMBINER_INDEXED:
            for (int i = 0; i < ints[0] && ok; i++)
                ok = flatten(types[0], ints[1 + i], at + (MPI_Aint)ints[1 + ints[0] + i] * ext0, out, depth + 1);
            break;
        case MPI_COMBINER_HINDEXED:
            for (int i = 0; i < ints[0] && ok; i++) ok = flatten(types[0], ints[1 + i], at + adds[i], out, depth + 1);
            break;
        case MPI_COMBINER_INDEXED_BLOCK:
            for (int i = 0; i < ints[0] && ok; i++)
                ok = flatten(types[0], ints[1], at + (MPI_Aint)ints[2 + i] * ext0, out, depth + 1);
            break;
        case MPI_COMBINER_HINDEXED_BLOCK:
            for (int i = 0; i < ints[0] && ok; i++) ok = flatten(types[0], ints[1], at + adds[i], out, depth + 1);
            break;
        case MPI_COMBINER_STRUCT:
            for (int i = 0; i < ints[0] && ok; i++) ok = flatten(types[i], ints[1 + i], at + adds[i], out, depth + 1);
            break;
        default: ok = false;
        }
    }
    for (MPI_Datatype& ty : types)
        if (!is_named(ty)) MPI_Type_free(&ty);
    return ok;
}

// Host-staged transport over MPI (dccrgx_host_transport) for ranks that
// share a GPU -- RCCL refuses two ranks on one device.  One update's
// messages go as the reference's transfer engine moves them: Irecv / Isend
// per peer, then Waitall (dccrg.hpp:10726-11209); scalars by MPI_Allreduce.
inline int mpi_exchange(void* user, int32_t ns, const int32_t* sp, const void* const* sb, const uint64_t* sn,
                        int32_t nr, const int32_t* rp, void* const* rb, const uint64_t* rn)
{
    const MPI_Comm comm = *static_cast<const MPI_Comm*>(user);
    // int counts: a message of 2 GiB or more goes as 1 GiB pieces in order
    // (same source, tag and communicator: MPI keeps them in order)
    const uint64_t piece = uint64_t(1) << 30;
    std::vector<MPI_Request> req;
    for (int32_t i = 0; i < nr; i++)
        for (uint64_t o = 0; o < rn[i]; o += piece) {
            req.push_back(MPI_REQUEST_NULL);
            const int cnt = (int)std::min<uint64_t>(piece, rn[i] - o);
            if (MPI_Irecv(static_cast<char*>(rb[i]) + o, cnt, MPI_BYTE, rp[i], 0, comm, &req.back()) != MPI_SUCCESS)
                return 1;
        }
    for (int32_t i = 0; i < ns; i++)
        for (uint64_t o = 0; o < sn[i]; o += piece) {
            req.push_back(MPI_REQUEST_NULL);
            const int cnt = (int)std::min<uint64_t>(piece, sn[i] - o);
            if (MPI_Isend(const_cast<char*>(static_cast<const char*>(sb[i])) + o, cnt, MPI_BYTE, sp[i], 0, comm,
                          &req.back()) != MPI_SUCCESS)
                return 1;
        }
    return MPI_Waitall((int)req.size(), req.data(), MPI_STATUSES_IGNORE) == MPI_SUCCESS ? 0 : 1;
}
inline int mpi_allreduce_f64(void* user, double* v, int32_t n, int32_t op)
{
    const MPI_Comm comm = *static_cast<const MPI_Comm*>(user);
    const MPI_Op o = op == 0 ? MPI_SUM : op == 1 ? MPI_MIN : MPI_MAX;
    return MPI_Allreduce(MPI_IN_PLACE, v, n, MPI_DOUBLE, o, comm) == MPI_SUCCESS ? 0 : 1;
}

}  // namespace detail

class Grid_Length {  // dccrg_length.hpp:34-142
public:
    typedef std::array<uint64_t, 3> type;
    const type& get() const { return l_; }
    type l_{{1, 1, 1}};
};

class Grid_Topology {  // dccrg_topology.hpp:38-217
public:
    bool is_periodic(size_t d) const { return d < 3 && p_[d]; }
    bool set_periodicity(size_t d, bool v)
    {
        if (d > 2) return false;
        p_[d] = v;
        return true;
    }
    std::array<bool, 3> p_{{false, false, false}};
};

// dccrg_mapping.hpp:55-690 (host-side scalar calls of libdccrgx)
class Mapping {
public:
    Grid_Length length;

    bool set_length(const Grid_Length::type& l)
    {
        if (!l[0] || !l[1] || !l[2]) return false;
        length.l_ = l;
        return true;
    }
    bool set_maximum_refinement_level(int lvl)
    {
        int maxp = 0;
        detail::check(dccrgx_max_possible_refinement_level(length.l_.data(), &maxp), "max level");
        if (lvl > maxp) return false;
        max_lvl_ = lvl < 0 ? maxp : lvl;
        return true;
    }
    const int& get_maximum_refinement_level() const { return max_lvl_; }
    int get_maximum_possible_refinement_level() const
    {
        int maxp = 0;
        detail::check(dccrgx_max_possible_refinement_level(length.l_.data(), &maxp), "max level");
        return maxp;
    }
    uint64_t get_last_cell() const
    {
        uint64_t v = 0;
        const dccrgx_mapping m = raw();
        detail::check(dccrgx_last_cell(&m, &v), "last cell");
        return v;
    }
    uint64_t get_cell_from_indices(const Types<3>::indices_t& idx, int lvl) const
    {
        uint64_t v = 0;
        const dccrgx_mapping m = raw();
        detail::check(dccrgx_map_host_cell(&m, idx.data(), lvl, &v), "get_cell_from_indices");
        return v;
    }
    Types<3>::indices_t get_indices(uint64_t cell) const
    {
        Types<3>::indices_t out;
        const dccrgx_mapping m = raw();
        detail::check(dccrgx_map_host_indices(&m, cell, out.data(), nullptr), "get_indices");
        return out;
    }
    int get_refinement_level(uint64_t cell) const
    {
        Types<3>::indices_t out;
        int32_t l = -1;
        const dccrgx_mapping m = raw();
        detail::check(dccrgx_map_host_indices(&m, cell, out.data(), &l), "get_refinement_level");
        return l;
    }
    uint64_t get_cell_length_in_indices(uint64_t c) const { return op(DCCRGX_OP_LENGTH_IN_INDICES, c); }
    uint64_t get_parent(uint64_t c) const { return op(DCCRGX_OP_PARENT, c); }
    uint64_t get_level_0_parent(uint64_t c) const { return op(DCCRGX_OP_LEVEL_0_PARENT, c); }
    uint64_t get_child(uint64_t c) const { return op(DCCRGX_OP_CHILD, c); }
    // dccrg_mapping.hpp:392-442, x fastest then y then z.  Like the reference,
    // an id beyond the last cell (level -1) is not rejected: its error_index
    // corner wraps in unsigned arithmetic (pinned by tests/golden/ref_mapping.npz)
    std::array<uint64_t, 8> get_all_children(uint64_t cell) const
    {
        std::array<uint64_t, 8> ch;
        ch.fill(error_cell);
        const int l = get_refinement_level(cell);
        if (cell == error_cell || l >= max_lvl_) return ch;
        const auto idx = get_indices(cell);
        const uint64_t off = uint64_t(1) << (max_lvl_ - l - 1);
        size_t i = 0;
        for (uint64_t z = 0; z < 2 * off; z += off)
            for (uint64_t y = 0; y < 2 * off; y += off)
                for (uint64_t x = 0; x < 2 * off; x += off)
                    ch[i++] = get_cell_from_indices({{idx[0] + x, idx[1] + y, idx[2] + z}}, l + 1);
        return ch;
    }
    std::array<uint64_t, 8> get_siblings(uint64_t cell) const  // dccrg_mapping.hpp:450-471
    {
        std::array<uint64_t, 8> s;
        s.fill(error_cell);
        const int l = get_refinement_level(cell);
        if (l < 0) return s;
        if (l == 0) {
            s[0] = cell;
            return s;
        }
        return get_all_children(get_parent(cell));
    }
    dccrgx_mapping raw() const
    {
        dccrgx_mapping m{};
        for (int d = 0; d < 3; d++) m.length[d] = length.l_[d];
        m.max_ref_lvl = max_lvl_;
        return m;
    }

private:
    uint64_t op(int o, uint64_t c) const
    {
        uint64_t v = 0;
        const dccrgx_mapping m = raw();
        detail::check(dccrgx_map_host_op(&m, o, c, &v), "mapping");
        return v;
    }
    int max_lvl_ = 0;
};

// dccrg_no_geometry.hpp: level-0 cells of unit length from the origin; its
// parameters are a dummy integer (:104-131)
struct No_Geometry {
    static const int geometry_id = 0;
    typedef int Parameters;
    explicit No_Geometry(const Mapping* m = nullptr, const Grid_Topology* t = nullptr) : mapping_(m), topology_(t) {}
    bool set(const Parameters&) { return true; }
    bool set(const No_Geometry&) { return true; }
    const Parameters& get() const { return par_; }
    std::array<double, 3> get_start() const { return {{0, 0, 0}}; }
    std::array<double, 3> get_end() const  // :155-168: the level-0 lengths
    {
        const auto& l = mapping_->length.get();
        return {{double(l[0]), double(l[1]), double(l[2])}};
    }
    std::array<double, 3> get_level_0_cell_length() const { return {{1, 1, 1}}; }
    // :183-206 (NaN for error_cell or an invalid cell)
    std::array<double, 3> get_length(uint64_t cell) const
    {
        const int l = mapping_->get_refinement_level(cell);
        if (cell == error_cell || l < 0 || l > mapping_->get_maximum_refinement_level()) return nan3();
        const double len = 1.0 / double(uint64_t(1) << l);
        return {{len, len, len}};
    }
    // :217-255: index / 2^max + length / 2
    std::array<double, 3> get_center(uint64_t cell) const
    {
        const int l = mapping_->get_refinement_level(cell);
        if (cell == error_cell || l < 0 || l > mapping_->get_maximum_refinement_level()) return nan3();
        const auto idx = mapping_->get_indices(cell);
        const auto len = get_length(cell);
        const double top = double(uint64_t(1) << mapping_->get_maximum_refinement_level());
        std::array<double, 3> c;
        for (int d = 0; d < 3; d++) c[d] = double(idx[d]) / top + len[d] / 2;
        return c;
    }
    std::array<double, 3> get_min(uint64_t cell) const  // :266-281
    {
        const auto c = get_center(cell), len = get_length(cell);
        return {{c[0] - len[0] / 2, c[1] - len[1] / 2, c[2] - len[2] / 2}};
    }
    std::array<double, 3> get_max(uint64_t cell) const  // :292-307
    {
        const auto c = get_center(cell), len = get_length(cell);
        return {{c[0] + len[0] / 2, c[1] + len[1] / 2, c[2] + len[2] / 2}};
    }
    // :313-360: the center of a cell of a level at maximum-level indices (an
    // index may equal the grid's end, as there)
    std::array<double, 3> get_center(int level, const Types<3>::indices_t& index) const
    {
        const int top_lvl = mapping_->get_maximum_refinement_level();
        if (level < 0 || level > top_lvl) return nan3();
        const uint64_t scale = uint64_t(1) << top_lvl;
        const auto& l = mapping_->length.get();
        for (int d = 0; d < 3; d++)
            if (index[d] > l[d] * scale) return nan3();
        const double half = 1.0 / double(uint64_t(1) << level) / 2;
        std::array<double, 3> c;
        for (int d = 0; d < 3; d++) c[d] = double(index[d]) / double(scale) + half;
        return c;
    }
    // :397-431: inside, its periodic image, or NaN
    std::array<double, 3> get_real_coordinate(const std::array<double, 3>& c) const
    {
        const std::array<double, 3> end = get_end();
        std::array<double, 3> r = nan3();
        for (int d = 0; d < 3; d++) {
            if (c[d] >= 0.0 && c[d] <= end[d]) {
                r[d] = c[d];
            } else if (topology_ && topology_->is_periodic(d)) {
                if (c[d] < 0.0) r[d] = c[d] + end[d] * std::ceil(-c[d] / end[d]);
                else r[d] = c[d] - end[d] * std::ceil((c[d] - end[d]) / end[d]);
            }
        }
        return r;
    }
    // :434-454: the floor of the (real) coordinate itself, error_index outside
    Types<3>::indices_t get_indices(const std::array<double, 3>& given) const
    {
        Types<3>::indices_t r{{error_index, error_index, error_index}};
        const std::array<double, 3> end = get_end(), c = get_real_coordinate(given);
        for (int d = 0; d < 3; d++)
            if (c[d] >= 0.0 && c[d] <= end[d]) r[d] = uint64_t(std::floor(c[d]));
        return r;
    }
    uint64_t get_cell(int level, const std::array<double, 3>& c) const  // :371-386
    {
        if (level < 0 || level > mapping_->get_maximum_refinement_level()) return error_cell;
        return mapping_->get_cell_from_indices(get_indices(c), level);
    }
    bool read_file_data(const std::vector<char>& b) const
    {
        int id = -1;
        if (b.size() < 4) return false;
        std::memcpy(&id, b.data(), 4);
        return id == geometry_id;
    }
    // file data, dccrg_no_geometry.hpp:486-549: the id
    std::vector<char> file_data() const
    {
        std::vector<char> b(4);
        const int id = geometry_id;
        std::memcpy(b.data(), &id, 4);
        return b;
    }

private:
    static std::array<double, 3> nan3()
    {
        const double q = std::numeric_limits<double>::quiet_NaN();
        return {{q, q, q}};
    }
    const Mapping* mapping_;
    const Grid_Topology* topology_;
    Parameters par_ = 0;
};

// dccrg_cartesian_geometry.hpp:51-812: level-0 cells of the same size from a
// starting corner; lengths and centers of any cell from the mapping
struct Cartesian_Geometry_Parameters {
    std::array<double, 3> start{{0, 0, 0}}, level_0_cell_length{{1, 1, 1}};
    Cartesian_Geometry_Parameters() = default;
    Cartesian_Geometry_Parameters(const std::array<double, 3>& s, const std::array<double, 3>& l)
        : start(s), level_0_cell_length(l)
    {
        for (double v : l)
            if (!(v > 0)) throw std::invalid_argument("level-0 cell length must be > 0");
    }
};

struct Cartesian_Geometry {
    static const int geometry_id = 1;
    typedef Cartesian_Geometry_Parameters Parameters;
    explicit Cartesian_Geometry(const Mapping* m = nullptr, const Grid_Topology* t = nullptr)
        : mapping_(m), topology_(t)
    {
    }
    bool set(const Parameters& p)
    {
        for (double v : p.level_0_cell_length)
            if (!(v > 0)) return false;
        par_ = p;
        return true;
    }
    const Parameters& get() const { return par_; }
    std::array<double, 3> get_start() const { return par_.start; }
    std::array<double, 3> get_level_0_cell_length() const { return par_.level_0_cell_length; }
    // :244-268: the corner with the largest coordinates
    std::array<double, 3> get_end() const
    {
        const auto& len = mapping_->length.get();
        std::array<double, 3> e;
        for (int d = 0; d < 3; d++) e[d] = par_.start[d] + double(len[d]) * par_.level_0_cell_length[d];
        return e;
    }
    // :522-566: the coordinate itself inside the grid, its periodic image
    // inside a periodic dimension, NaN outside a non-periodic one
    std::array<double, 3> get_real_coordinate(const std::array<double, 3>& c) const
    {
        const std::array<double, 3> start = par_.start, end = get_end();
        std::array<double, 3> r = nan3();
        for (int d = 0; d < 3; d++) {
            if (c[d] >= start[d] && c[d] <= end[d]) {
                r[d] = c[d];
            } else if (topology_ && topology_->is_periodic(d)) {
                const double L = end[d] - start[d];
                if (c[d] < start[d]) r[d] = c[d] + L * std::ceil((start[d] - c[d]) / L);
                else r[d] = c[d] - L * std::ceil((c[d] - end[d]) / L);
            }
        }
        return r;
    }
    // :576-608: indices (maximum-level units) of a coordinate, error_index
    // outside a non-periodic dimension
    Types<3>::indices_t get_indices(const std::array<double, 3>& given) const
    {
        Types<3>::indices_t r{{error_index, error_index, error_index}};
        const std::array<double, 3> start = par_.start, end = get_end(), c = get_real_coordinate(given);
        const double top = double(uint64_t(1) << mapping_->get_maximum_refinement_level());
        for (int d = 0; d < 3; d++)
            if (c[d] >= start[d] && c[d] <= end[d])
                r[d] = uint64_t(std::floor((c[d] - start[d]) / (par_.level_0_cell_length[d] / top)));
        return r;
    }
    // :496-507: the cell of a refinement level at a coordinate
    uint64_t get_cell(int level, const std::array<double, 3>& c) const
    {
        if (level < 0 || level > mapping_->get_maximum_refinement_level()) return error_cell;
        return mapping_->get_cell_from_indices(get_indices(c), level);
    }
    // :284-309 (NaN for error_cell or an invalid cell)
    std::array<double, 3> get_length(uint64_t cell) const
    {
        const int l = mapping_->get_refinement_level(cell);
        if (cell == error_cell || l < 0 || l > mapping_->get_maximum_refinement_level()) return nan3();
        const double f = 1.0 / double(uint64_t(1) << l);
        return {{par_.level_0_cell_length[0] * f, par_.level_0_cell_length[1] * f, par_.level_0_cell_length[2] * f}};
    }
    // :318-364: start + index * l0 / 2^max + length / 2, in that order
    std::array<double, 3> get_center(uint64_t cell) const
    {
        const int l = mapping_->get_refinement_level(cell);
        if (cell == error_cell || l < 0 || l > mapping_->get_maximum_refinement_level()) return nan3();
        const auto idx = mapping_->get_indices(cell);
        const auto len = get_length(cell);
        const double top = double(uint64_t(1) << mapping_->get_maximum_refinement_level());
        std::array<double, 3> c;
        for (int d = 0; d < 3; d++) c[d] = par_.start[d] + double(idx[d]) * par_.level_0_cell_length[d] / top + len[d] / 2;
        return c;
    }
    std::array<double, 3> get_min(uint64_t cell) const  // :378-400
    {
        const auto c = get_center(cell), len = get_length(cell);
        return {{c[0] - len[0] / 2, c[1] - len[1] / 2, c[2] - len[2] / 2}};
    }
    std::array<double, 3> get_max(uint64_t cell) const  // :404-422
    {
        const auto c = get_center(cell), len = get_length(cell);
        return {{c[0] + len[0] / 2, c[1] + len[1] / 2, c[2] + len[2] / 2}};
    }
    bool read_file_data(const std::vector<char>& b)  // :683-756
    {
        int id = -1;
        if (b.size() < 52) return false;
        std::memcpy(&id, b.data(), 4);
        if (id != geometry_id) return false;
        Parameters p;
        std::memcpy(p.start.data(), b.data() + 4, 24);
        std::memcpy(p.level_0_cell_length.data(), b.data() + 28, 24);
        return set(p);
    }
    // file data, :620-680: id, start, level-0 cell length
    std::vector<char> file_data() const
    {
        std::vector<char> b(4 + 48);
        const int id = geometry_id;
        std::memcpy(b.data(), &id, 4);
        std::memcpy(b.data() + 4, par_.start.data(), 24);
        std::memcpy(b.data() + 28, par_.level_0_cell_length.data(), 24);
        return b;
    }

private:
    static std::array<double, 3> nan3()
    {
        const double q = std::numeric_limits<double>::quiet_NaN();
        return {{q, q, q}};
    }
    const Mapping* mapping_;
    const Grid_Topology* topology_ = nullptr;
    Parameters par_;
};

template <class Cell_Data, class Geometry = No_Geometry, class Additional_Cell_Items = std::tuple<>,
          class Additional_Neighbor_Items = std::tuple<>>
class Dccrg;

// Additional cell / neighbor items (dccrg.hpp:151-156, 7404-7518): the
// iteration cache's items derive from them, and each item's update() is
// called when the cache is (re)built, as update_caller does (:11548, 11650)
template <class Cell_Data, class Geometry, class... ACI, class... ANI>
class Dccrg<Cell_Data, Geometry, std::tuple<ACI...>, std::tuple<ANI...>> {
public:
    typedef std::vector<std::pair<uint64_t, std::array<int, 3>>> neighbor_list_t;

    // dccrg.hpp:7394-7401
    template <class T> struct Iterator_Storage {
        typename std::vector<T>::const_iterator begin_, end_;
        typename std::vector<T>::const_iterator begin() const { return begin_; }
        typename std::vector<T>::const_iterator cbegin() const { return begin_; }
        typename std::vector<T>::const_iterator end() const { return end_; }
        typename std::vector<T>::const_iterator cend() const { return end_; }
    };
    struct Neighbors_Item : ANI... {  // dccrg.hpp:7404-7456
        uint64_t id = error_cell;
        Cell_Data* data = nullptr;
        int x = 0, y = 0, z = 0;
    };
    struct Cells_Item : ACI... {  // dccrg.hpp:7480-7518
        uint64_t id = error_cell;
        Cell_Data* data = nullptr;
        Iterator_Storage<Neighbors_Item> neighbors_of, neighbors_to, all_neighbors;
    };

    Mapping mapping;
    Grid_Topology topology;
    Geometry geometry{&mapping, &topology};

    // dccrg.hpp:7547 (const std::vector<Cells_Item>& cells): every cell of the
    // default neighborhood's iteration cache, local then copies of remote
    // ones; a read-only view here, since the cache is rebuilt in place
    class Cells_View {
    public:
        typedef typename std::vector<Cells_Item>::const_iterator const_iterator;
        explicit Cells_View(const Dccrg* g) : g_(g) {}
        const std::vector<Cells_Item>& get() const
        {
            static const std::vector<Cells_Item> none;
            const auto it = g_->hoods_.find(default_neighborhood_id);
            return it == g_->hoods_.end() ? none : it->second.cells;
        }
        operator const std::vector<Cells_Item>&() const { return get(); }
        const_iterator begin() const { return get().begin(); }
        const_iterator end() const { return get().end(); }
        const_iterator cbegin() const { return get().begin(); }
        const_iterator cend() const { return get().end(); }
        size_t size() const { return get().size(); }
        bool empty() const { return get().empty(); }
        const Cells_Item& operator[](size_t i) const { return get()[i]; }
        const Cells_Item& at(size_t i) const { return get().at(i); }

    private:
        const Dccrg* g_;
    };
    const Cells_View cells{this};

    Dccrg() = default;
    Dccrg(const Dccrg&) = delete;
    // dccrg.hpp:327-446: a grid of another cell data type over the same cells,
    // owners, neighborhoods (user ones included), cell weights and
    // communicator, already initialized; the local cells' data is
    // default-constructed and the copies of remote neighbors allocated.  Cell
    // owners follow the level-0 ancestors here (no load balancing moves a
    // cell), so the same leaves under the same partition give the same owners.
    template <class O_Cell, class O_Geometry, class O_ACI, class O_ANI>
    explicit Dccrg(const Dccrg<O_Cell, O_Geometry, O_ACI, O_ANI>& other)
    {
        if (!other.get_initialized()) throw std::invalid_argument("copy of a grid that is not initialized");
        mapping.set_length(other.mapping.length.get());
        mapping.set_maximum_refinement_level(other.mapping.get_maximum_refinement_level());
        for (int d = 0; d < 3; d++) topology.set_periodicity(d, other.topology.is_periodic(d));
        if (!copy_geometry(other.geometry)) throw std::invalid_argument("geometry of the other grid not accepted");
        hood_length_ = other.get_neighborhood_length();
        send_single_cells_ = other.get_send_single_cells();
        partition_ = (uint8_t)other.get_initial_partition();
        init_comm(other.get_communicator());
        dccrgx_grid_params p{};
        for (int d = 0; d < 3; d++) {
            p.length[d] = mapping.length.get()[d];
            p.periodic[d] = topology.is_periodic(d) ? 1 : 0;
        }
        p.max_ref_lvl = mapping.get_maximum_refinement_level();
        p.neighborhood_length = hood_length_;
        p.partition = partition_;
        // every level-0 cell and nothing else: keep the uniform layout
        const std::vector<uint64_t> leaves = other.get_all_cells();
        const uint64_t n0 = p.length[0] * p.length[1] * p.length[2];
        const bool level0 = leaves.size() == n0 && (n0 == 0 || leaves.back() == n0);
        detail::check(dccrgx_grid_create(ctx_, &p, level0 ? nullptr : leaves.data(), level0 ? 0 : leaves.size(),
                                         &grid_),
                      "grid");
        for (uint64_t c : query_cells(default_neighborhood_id, DCCRGX_CELLS_LOCAL)) cell_data_[c];
        cell_weights_ = other.get_cell_weights();
        initialized_ = true;
        build_hood(default_neighborhood_id);
        for (const auto& kv : other.get_user_hood_of())
            if (!add_neighborhood(kv.first, kv.second)) throw std::invalid_argument("neighborhood of the other grid");
    }
    ~Dccrg()
    {
        if (grid_) dccrgx_grid_destroy(grid_);
        if (ctx_) dccrgx_ctx_destroy(ctx_);
        if (comm_ != MPI_COMM_NULL) {
            int fin = 0;
            MPI_Finalized(&fin);
            if (!fin) MPI_Comm_free(&comm_);
        }
    }

    // ---- configuration (dccrg.hpp:8242-8361) ------------------------------
    Dccrg& set_initial_length(const std::array<uint64_t, 3>& l)
    {
        if (initialized_) throw std::invalid_argument("set_initial_length after initialize");
        if (!mapping.set_length(l)) throw std::invalid_argument("all lengths must be > 0");
        return *this;
    }
    Dccrg& set_maximum_refinement_level(int lvl)
    {
        if (initialized_) throw std::invalid_argument("set_maximum_refinement_level after initialize");
        if (!mapping.set_maximum_refinement_level(lvl)) throw std::invalid_argument("refinement level too large");
        return *this;
    }
    Dccrg& set_periodic(bool x, bool y, bool z)
    {
        if (initialized_) throw std::invalid_argument("set_periodic after initialize");
        topology.set_periodicity(0, x);
        topology.set_periodicity(1, y);
        topology.set_periodicity(2, z);
        return *this;
    }
    Dccrg& set_neighborhood_length(unsigned n)
    {
        if (initialized_) throw std::invalid_argument("set_neighborhood_length after initialize");
        hood_length_ = n;
        return *this;
    }
    Dccrg& set_load_balancing_method(const std::string&) { return *this; }
    // placement of the level-0 cells (create_level_0_cells, dccrg.hpp:8089-8224):
    // DCCRGX_PARTITION_BLOCK (the default build) or DCCRGX_PARTITION_SFC (what
    // the reference selects at compile time with USE_SFC, :8147-8220)
    Dccrg& set_initial_partition(int partition)
    {
        if (initialized_) throw std::invalid_argument("set_initial_partition after initialize");
        if (partition != DCCRGX_PARTITION_BLOCK && partition != DCCRGX_PARTITION_SFC)
            throw std::invalid_argument("unknown partition");
        partition_ = (uint8_t)partition;
        return *this;
    }
    // dccrg.hpp:586-595: chained; throws when the geometry rejects the parameters
    Dccrg& set_geometry(const typename Geometry::Parameters& p)
    {
        if (!geometry.set(p)) throw std::invalid_argument("Couldn't set geometry");
        return *this;
    }
    int get_initial_partition() const { return partition_; }
    // dccrg.hpp:1046-1064 as built with DCCRG_NO_LB (Zoltan stays out of the
    // device path): the body is compiled out, so nothing moves and the
    // iteration caches, additional items and references into `cells` stay
    // as they are
    Dccrg& balance_load(bool = true) { return *this; }
    // facade extension, not in the reference: rebuild the iteration caches
    // and run the additional items' update() again -- what a Zoltan build's
    // balance_load does through update_cell_pointers (:4130-4144, :11453),
    // e.g. to refresh a Center item after set_geometry.  Invalidates
    // references into `cells`.
    Dccrg& refresh_additional_items()
    {
        if (!initialized_) return *this;
        std::vector<int> ids;
        for (auto& kv : hoods_) ids.push_back(kv.first);
        for (int id : ids) build_hood(id);
        return *this;
    }

    // dccrg.hpp:485-562
    Dccrg& initialize(const MPI_Comm& comm, uint64_t = 1)
    {
        if (initialized_) throw std::invalid_argument("already initialized");
        init_comm(comm);
        dccrgx_grid_params p{};
        for (int d = 0; d < 3; d++) {
            p.length[d] = mapping.length.get()[d];
            p.periodic[d] = topology.is_periodic(d) ? 1 : 0;
        }
        p.max_ref_lvl = mapping.get_maximum_refinement_level();
        p.neighborhood_length = hood_length_;
        p.partition = partition_;
        detail::check(dccrgx_grid_create(ctx_, &p, nullptr, 0, &grid_), "grid");
        for (uint64_t c : query_cells(default_neighborhood_id, DCCRGX_CELLS_LOCAL)) cell_data_[c];
        initialized_ = true;
        build_hood(default_neighborhood_id);
        return *this;
    }

    // ---- grid data files (dccrg.hpp:1109-2427) -------------------------------
    // save_grid_data: the header's packed bytes (rank 0), then the layout of
    // include/dccrgx.h; every cell's record is the packed form of its
    // get_mpi_datatype(id, rank, -1, false, -1) (:1324-1340).  Collective.
    bool save_grid_data(const std::string& name, MPI_Offset offset, std::tuple<void*, int, MPI_Datatype> header)
    {
        const std::vector<char> hb = pack_header(header);
        const std::vector<uint64_t> ids = get_cells();
        std::vector<uint64_t> sizes;
        std::vector<char> recs;
        for (uint64_t c : ids) {
            const size_t before = recs.size();
            pack(c, cell_data_.at(c), rank_, -1, false, -1, recs);
            sizes.push_back(recs.size() - before);
        }
        uint64_t mine[2] = {ids.size(), recs.size()};
        std::vector<uint64_t> all(2 * size_);
        MPI_Allgather(mine, 2, MPI_UINT64_T, all.data(), 2, MPI_UINT64_T, comm_);
        uint64_t total = 0, cells_before = 0, bytes_before = 0;
        for (int r = 0; r < size_; r++) {
            total += all[2 * r];
            if (r < rank_) {
                cells_before += all[2 * r];
                bytes_before += all[2 * r + 1];
            }
        }
        const std::vector<char> gb = geometry.file_data();  // the geometry's write(), e.g. :620-680
        const int s = dccrgx_save_grid_data_host(grid_, name.c_str(), (uint64_t)offset, hb.data(), hb.size(),
                                                 gb.data(), gb.size(), total, cells_before, bytes_before, sizes.data(),
                                                 recs.data(), recs.size());
        int ok = s == DCCRGX_OK, all_ok = 0;
        if (!ok) std::fprintf(stderr, "save_grid_data: %s\n", dccrgx_last_error());
        MPI_Allreduce(&ok, &all_ok, 1, MPI_INT, MPI_MIN, comm_);
        return all_ok != 0;
    }
    bool load_grid_data(const std::string& name, MPI_Offset offset, std::tuple<void*, int, MPI_Datatype> header,
                        const MPI_Comm& comm, const char* load_balancing_method, uint64_t sfc_caching_batches = 1,
                        uint64_t number_of_cells = ~uint64_t(0))
    {
        return start_loading_grid_data(name, offset, header, comm, load_balancing_method, sfc_caching_batches,
                                       number_of_cells) &&
               continue_loading_grid_data() && finish_loading_grid_data();
    }
    // dccrg.hpp:1815-2105: creates the grid of the file's cells (instead of initialize())
    bool start_loading_grid_data(const std::string& name, MPI_Offset offset,
                                 std::tuple<void*, int, MPI_Datatype> header, const MPI_Comm& comm, const char*,
                                 uint64_t = 1, uint64_t = ~uint64_t(0))
    {
        if (initialized_) throw std::invalid_argument("already initialized");
        init_comm(comm);
        std::vector<char> hb(pack_header(header).size());
        dccrgx_file_info info{};
        std::vector<char> gb(4096);
        if (dccrgx_file_read_info(name.c_str(), (uint64_t)offset, hb.data(), hb.size(), &info, gb.data(), gb.size()) !=
            DCCRGX_OK) {
            std::fprintf(stderr, "start_loading_grid_data: %s\n", dccrgx_last_error());
            return false;
        }
        gb.resize(std::min<size_t>(gb.size(), info.geometry_bytes));
        if (!geometry.read_file_data(gb)) {
            std::fprintf(stderr, "start_loading_grid_data: the file's geometry is not this grid's geometry\n");
            return false;
        }
        int pos = 0;
        MPI_Datatype t = std::get<2>(header);
        const bool named = detail::is_named(t);
        if (!named) MPI_Type_commit(&t);
        if (!hb.empty()) MPI_Unpack(hb.data(), (int)hb.size(), &pos, std::get<0>(header), std::get<1>(header), t, comm_);
        if (!named) MPI_Type_free(&t);
        mapping.set_length({{info.params.length[0], info.params.length[1], info.params.length[2]}});
        mapping.set_maximum_refinement_level(info.params.max_ref_lvl);
        for (int d = 0; d < 3; d++) topology.set_periodicity(d, info.params.periodic[d] != 0);
        hood_length_ = info.params.neighborhood_length;
        if (dccrgx_grid_load(ctx_, name.c_str(), &info, &grid_) != DCCRGX_OK) {
            std::fprintf(stderr, "start_loading_grid_data: %s\n", dccrgx_last_error());
            return false;
        }
        for (uint64_t c : query_cells(default_neighborhood_id, DCCRGX_CELLS_LOCAL)) cell_data_[c];
        initialized_ = true;
        build_hood(default_neighborhood_id);
        return true;
    }
    // dccrg.hpp:2134-2390: each local cell's next bytes, as its
    // get_mpi_datatype(id, -1, rank, true, -1) describes them
    bool continue_loading_grid_data()
    {
        const std::vector<uint64_t> ids = get_cells();
        std::vector<uint64_t> sizes;
        uint64_t tot = 0;
        for (uint64_t c : ids) {
            sizes.push_back((uint64_t)pack_size(c, cell_data_.at(c), -1, rank_, true, -1));
            tot += sizes.back();
        }
        std::vector<char> buf(tot);
        if (dccrgx_load_cell_records_host(grid_, sizes.data(), buf.data(), buf.size()) != DCCRGX_OK) {
            std::fprintf(stderr, "continue_loading_grid_data: %s\n", dccrgx_last_error());
            return false;
        }
        int pos = 0;
        for (uint64_t c : ids) unpack(c, cell_data_.at(c), -1, rank_, -1, buf, pos);
        return true;
    }
    bool finish_loading_grid_data()  // dccrg.hpp:2402-2426
    {
        return dccrgx_finish_loading_grid_data(grid_) == DCCRGX_OK;
    }

private:
    // the converting constructor's geometry: the parameters of the same
    // geometry type, the default of this one otherwise
    bool copy_geometry(const Geometry& g) { return geometry.set(g.get()); }
    template <class G> bool copy_geometry(const G&) { return true; }
    void init_comm(const MPI_Comm& comm)
    {
        MPI_Comm_dup(comm, &comm_);
        MPI_Comm_rank(comm_, &rank_);
        MPI_Comm_size(comm_, &size_);
        MPI_Comm node;
        MPI_Comm_split_type(comm_, MPI_COMM_TYPE_SHARED, rank_, MPI_INFO_NULL, &node);
        int node_rank = 0, node_size = 1, ndev = 0;
        MPI_Comm_rank(node, &node_rank);
        MPI_Comm_size(node, &node_size);
        MPI_Comm_free(&node);
        detail::check(dccrgx_device_count(&ndev), "device count");
        if (ndev < 1) throw std::runtime_error("no GPU");
        detail::check(dccrgx_ctx_create(node_rank % ndev, rank_, size_, &ctx_), "context");
        int shared = node_size > ndev ? 1 : 0, any_shared = 0;  // one transport for every rank
        MPI_Allreduce(&shared, &any_shared, 1, MPI_INT, MPI_MAX, comm_);
        if (size_ > 1 && any_shared) {
            // more ranks than GPUs on this node: ranks share a device, which
            // RCCL refuses, so halos go through the host over MPI
            dccrgx_host_transport t;
            t.user = &comm_;
            t.exchange = &detail::mpi_exchange;
            t.allreduce_f64 = &detail::mpi_allreduce_f64;
            detail::check(dccrgx_ctx_set_host_transport(ctx_, &t), "host transport");
        } else if (size_ > 1) {
            uint8_t uid[128] = {0};
            if (rank_ == 0) detail::check(dccrgx_get_unique_id(uid), "unique id");
            MPI_Bcast(uid, 128, MPI_BYTE, 0, comm_);
            detail::check(dccrgx_ctx_comm_init(ctx_, uid), "RCCL communicator");
        }
    }
    std::vector<char> pack_header(std::tuple<void*, int, MPI_Datatype> header) const
    {
        MPI_Datatype t = std::get<2>(header);
        const bool named = detail::is_named(t);
        if (!named) MPI_Type_commit(&t);
        int sz = 0;
        MPI_Pack_size(std::get<1>(header), t, comm_, &sz);
        std::vector<char> b(sz);
        int pos = 0;
        if (sz) MPI_Pack(std::get<0>(header), std::get<1>(header), t, b.data(), sz, &pos, comm_);
        b.resize(pos);
        if (!named) MPI_Type_free(&t);
        return b;
    }

public:
    // ---- queries ------------------------------------------------------------
    int get_rank() const { return rank_; }
    int get_comm_size() const { return size_; }
    MPI_Comm get_communicator() const { return comm_; }
    int get_maximum_refinement_level() const { return mapping.get_maximum_refinement_level(); }
    unsigned get_neighborhood_length() const { return hood_length_; }
    const Grid_Length& length() const { return mapping.length; }

    // dccrg.hpp:768-781: local cells, copies of remote neighbors, then data
    // of refined / unrefined cells (until clear_refined_unrefined_data)
    Cell_Data* operator[](uint64_t cell) const
    {
        for (const auto* m : {&cell_data_, &remote_data_, &refined_data_, &unrefined_data_}) {
            auto it = m->find(cell);
            if (it != m->end()) return const_cast<Cell_Data*>(&it->second);
        }
        return nullptr;
    }

    // ---- adaptive mesh refinement (dccrg.hpp:2456-2806, 3483-3543, 5550-5567)
    bool refine_completely(uint64_t cell) { return request(dccrgx_refine_completely, cell); }
    bool unrefine_completely(uint64_t cell) { return request(dccrgx_unrefine_completely, cell); }
    bool dont_refine(uint64_t cell) { return request(dccrgx_dont_refine, cell); }
    bool dont_unrefine(uint64_t cell) { return request(dccrgx_dont_unrefine, cell); }
    // dccrg.hpp:5905-6130 as built with DCCRG_NO_LB (load balancing is not on
    // this path: the partition stays the block one): pins do nothing
    bool pin(uint64_t) { return false; }
    bool pin(uint64_t, int) { return false; }
    bool unpin(uint64_t) { return false; }
    bool unpin_local_cells() { return false; }
    Dccrg& unpin_all_cells() { return *this; }
    // dccrg.hpp:6318-6379, 6450-6462: weights of local leaves (1 when unset),
    // inherited by the children of a refined cell (:10392-10398), dropped with
    // unrefined cells (:10509)
    bool set_cell_weight(uint64_t cell, double weight)
    {
        if (!is_local(cell)) return false;
        cell_weights_[cell] = weight;
        return true;
    }
    double get_cell_weight(uint64_t cell) const
    {
        if (!is_local(cell)) return std::numeric_limits<double>::quiet_NaN();
        auto it = cell_weights_.find(cell);
        return it == cell_weights_.end() ? 1.0 : it->second;
    }
    const std::unordered_map<uint64_t, double>& get_cell_weights() const { return cell_weights_; }
    // dccrg.hpp:3401-3467: the same for the smallest existing cell at a coordinate
    bool refine_completely_at(const std::array<double, 3>& c)
    {
        const uint64_t cell = get_existing_cell(c);
        return cell != error_cell && refine_completely(cell);
    }
    bool unrefine_completely_at(const std::array<double, 3>& c)
    {
        const uint64_t cell = get_existing_cell(c);
        return cell != error_cell && unrefine_completely(cell);
    }
    bool dont_unrefine_at(const std::array<double, 3>& c)
    {
        const uint64_t cell = get_existing_cell(c);
        return cell != error_cell && dont_unrefine(cell);
    }
    // dccrg.hpp:11414-11447: the smallest existing cell at the indices between
    // two refinement levels inclusive, else error_cell
    uint64_t get_existing_cell(const Types<3>::indices_t& idx, int min_level, int max_level) const
    {
        const int M = mapping.get_maximum_refinement_level();
        for (int d = 0; d < 3; d++)
            if (idx[d] >= mapping.length.get()[d] * (uint64_t(1) << M)) return error_cell;
        if (min_level > max_level) return error_cell;
        for (int l = max_level; l >= min_level; l--) {
            const uint64_t cell = mapping.get_cell_from_indices(idx, l);
            if (cell != error_cell && get_process(cell) >= 0) return cell;
        }
        return error_cell;
    }
    // dccrg.hpp:6424-6444: ... at a coordinate (the geometry's indices)
    uint64_t get_existing_cell(const std::array<double, 3>& c) const
    {
        const Types<3>::indices_t idx = geometry.get_indices(c);
        if (idx[0] == error_index || idx[1] == error_index || idx[2] == error_index) return error_cell;
        return get_existing_cell(idx, 0, mapping.get_maximum_refinement_level());
    }
    // dccrg.hpp:6752-6755: the largest refinement level difference between neighbors
    int get_max_ref_lvl_diff() const { return 1; }
    // dccrg.hpp:6717-6728
    bool get_initialized() const { return initialized_; }
    bool get_mapping_initialized() const { return true; }

    // collective; returns the cells created on this rank
    std::vector<uint64_t> stop_refining(bool sorted = false)
    {
        std::vector<uint64_t> sets[4];
        for (int k = 0; k < 4; k++) {
            size_t n = 0;
            detail::check(dccrgx_amr_requests(grid_, k, nullptr, 0, &n), "amr_requests");
            std::vector<uint64_t> mine(n);
            detail::check(dccrgx_amr_requests(grid_, k, mine.data(), n, &n), "amr_requests");
            int cnt = (int)n;
            std::vector<int> counts(size_), displs(size_, 0);
            MPI_Allgather(&cnt, 1, MPI_INT, counts.data(), 1, MPI_INT, comm_);
            for (int r = 1; r < size_; r++) displs[r] = displs[r - 1] + counts[r - 1];
            sets[k].resize((size_t)displs[size_ - 1] + counts[size_ - 1]);
            MPI_Allgatherv(mine.data(), cnt, MPI_UINT64_T, sets[k].data(), counts.data(), displs.data(),
                           MPI_UINT64_T, comm_);
            std::sort(sets[k].begin(), sets[k].end());
            sets[k].erase(std::unique(sets[k].begin(), sets[k].end()), sets[k].end());
        }
        const uint64_t* ptrs[4] = {sets[0].data(), sets[1].data(), sets[2].data(), sets[3].data()};
        const size_t counts[4] = {sets[0].size(), sets[1].size(), sets[2].size(), sets[3].size()};
        size_t n_new = 0;
        // every rank must reach the same leaf set: each builds its new grid
        // aside, the statuses are all-reduced, and all ranks adopt theirs or
        // all keep the old grid with the requests pending
        const int st = dccrgx_stop_refining_prepare(grid_, ptrs, counts, &n_new);
        const std::string err = st == DCCRGX_OK ? std::string() : std::string(dccrgx_last_error());
        int ok = st == DCCRGX_OK ? 1 : 0, all_ok = 0;
        MPI_Allreduce(&ok, &all_ok, 1, MPI_INT, MPI_MIN, comm_);
        detail::check(dccrgx_stop_refining_finish(grid_, all_ok), "stop_refining_finish");
        if (!all_ok)
            throw std::runtime_error(std::string("stop_refining failed on ") + (ok ? "another rank" : "this rank: ") +
                                     err + "; the grid is unchanged and the requests stay pending");
        std::vector<uint64_t> created = id_list(dccrgx_get_new_cells);
        // data moves as execute_refines moves it (dccrg.hpp:10266-10267,
        // 10354-10375, 10526-10590): previous refined/unrefined data dropped,
        // local cells that stopped being leaves kept aside, new cells
        // value-initialised
        refined_data_.clear();
        unrefined_data_.clear();
        const std::vector<uint64_t> removed = id_list(dccrgx_get_removed_cells);
        const std::unordered_set<uint64_t> removed_set(removed.begin(), removed.end());
        const std::vector<uint64_t> local = get_cells();
        const std::unordered_set<uint64_t> now(local.begin(), local.end());
        for (auto it = cell_data_.begin(); it != cell_data_.end();) {
            if (now.count(it->first)) {
                ++it;
                continue;
            }
            (removed_set.count(it->first) ? unrefined_data_ : refined_data_)[it->first] = std::move(it->second);
            it = cell_data_.erase(it);
        }
        for (uint64_t c : local) cell_data_[c];
        for (uint64_t c : created) {  // children of a refined local cell inherit its weight
            const uint64_t parent = mapping.get_cell_from_indices(mapping.get_indices(c),
                                                                  mapping.get_refinement_level(c) - 1);
            auto w = cell_weights_.find(parent);
            if (w != cell_weights_.end() && refined_data_.count(parent)) cell_weights_[c] = w->second;
        }
        for (auto it = cell_weights_.begin(); it != cell_weights_.end();)  // weights of cells that are gone
            it = now.count(it->first) ? std::next(it) : cell_weights_.erase(it);
        remote_data_.clear();
        std::vector<int> ids;
        for (auto& kv : hoods_) ids.push_back(kv.first);
        hoods_.clear();
        for (int id : ids) build_hood(id);
        if (sorted) std::sort(created.begin(), created.end());
        return created;
    }
    std::vector<uint64_t> get_removed_cells(bool sorted = false) const
    {
        std::vector<uint64_t> v;
        for (auto& kv : unrefined_data_) v.push_back(kv.first);
        if (sorted) std::sort(v.begin(), v.end());
        return v;
    }
    void clear_refined_unrefined_data()
    {
        detail::check(dccrgx_clear_refined_unrefined_data(grid_), "clear_refined_unrefined_data");
        refined_data_.clear();
        unrefined_data_.clear();
    }
    int get_refinement_level(uint64_t cell) const { return mapping.get_refinement_level(cell); }
    bool is_local(uint64_t cell) const { return cell_data_.count(cell) > 0; }
    // dccrg.hpp:5886-5902: the owning process of an existing cell, else -1
    int get_process(uint64_t cell) const
    {
        int32_t p = -1;
        detail::check(dccrgx_get_process(grid_, &cell, 1, &p), "get_process");
        return p;
    }
    // dccrg.hpp:4193-4226: the parent if it exists, else the cell if it
    // exists, else error_cell
    uint64_t get_parent(uint64_t cell) const
    {
        if (mapping.get_refinement_level(cell) == 0) return get_process(cell) >= 0 ? cell : error_cell;
        const uint64_t parent =
            mapping.get_cell_from_indices(mapping.get_indices(cell), mapping.get_refinement_level(cell) - 1);
        if (get_process(parent) >= 0) return parent;
        if (get_process(cell) >= 0) return cell;
        return error_cell;
    }

    // dccrg.hpp:661-742 / is_neighbor_type_match :2960-3081: local cells whose
    // neighbor types (has_*_neighbor_* of the neighborhood's neighbors_of and
    // neighbors_to) match the criteria; nothing for an unknown neighborhood.
    // Cells come ascending (the reference: hash order unless sorted).
    std::vector<uint64_t> get_cells(const std::vector<int>& criteria = std::vector<int>(), bool exact_match = false,
                                    int hood = default_neighborhood_id, bool /*sorted*/ = false) const
    {
        if (!hoods_.count(hood)) return {};
        std::vector<uint64_t> local = query_cells(hood, DCCRGX_CELLS_LOCAL);
        if (criteria.empty()) return local;
        const HoodState& S = hs(hood);
        std::vector<uint64_t> out;
        int merged = 0;
        for (int c : criteria) merged |= c;
        for (uint64_t cell : local) {
            int types = 0;
            for (const auto& n : S.nof.at(cell))
                if (n.first != error_cell) types |= is_local(n.first) ? has_local_neighbor_of : has_remote_neighbor_of;
            for (const auto& n : S.nto.at(cell))
                if (n.first != error_cell) types |= is_local(n.first) ? has_local_neighbor_to : has_remote_neighbor_to;
            bool match = false;
            if (exact_match) {
                for (int c : criteria) match |= types == c;
            } else {
                match = (types & merged) > 0;
            }
            if (match) out.push_back(cell);
        }
        return out;
    }
    // dccrg.hpp:6158-6300 (ascending; the reference: hash order unless sorted)
    std::vector<uint64_t> get_local_cells_on_process_boundary(int hood = default_neighborhood_id, bool = false) const
    {
        return hoods_.count(hood) ? query_cells(hood, DCCRGX_CELLS_OUTER) : std::vector<uint64_t>();
    }
    std::vector<uint64_t> get_local_cells_not_on_process_boundary(int hood = default_neighborhood_id, bool = false) const
    {
        return hoods_.count(hood) ? query_cells(hood, DCCRGX_CELLS_INNER) : std::vector<uint64_t>();
    }

    const Iterator_Storage<Cells_Item>& local_cells(int hood = default_neighborhood_id) const { return hs(hood).local; }
    const Iterator_Storage<Cells_Item>& inner_cells(int hood = default_neighborhood_id) const { return hs(hood).inner; }
    const Iterator_Storage<Cells_Item>& outer_cells(int hood = default_neighborhood_id) const { return hs(hood).outer; }
    const Iterator_Storage<Cells_Item>& remote_cells(int hood = default_neighborhood_id) const { return hs(hood).remote; }
    const Iterator_Storage<Cells_Item>& all_cells(int hood = default_neighborhood_id) const { return hs(hood).all; }

    // dccrg.hpp:836-883 / 900-943
    const neighbor_list_t* get_neighbors_of(uint64_t cell, int hood = default_neighborhood_id) const
    {
        auto h = hoods_.find(hood);
        if (h == hoods_.end()) return nullptr;
        auto it = h->second.nof.find(cell);
        return it == h->second.nof.end() ? nullptr : &it->second;
    }
    const neighbor_list_t* get_neighbors_to(uint64_t cell, int hood = default_neighborhood_id) const
    {
        auto h = hoods_.find(hood);
        if (h == hoods_.end()) return nullptr;
        auto it = h->second.nto.find(cell);
        return it == h->second.nto.end() ? nullptr : &it->second;
    }

    // dccrg.hpp:7008-7046: per process, ascending ids with tags 1..N
    const std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>& get_cells_to_send() const
    {
        return hs(default_neighborhood_id).send_tagged;
    }
    const std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>& get_cells_to_receive() const
    {
        return hs(default_neighborhood_id).recv_tagged;
    }
    // dccrg.hpp:5428-5536: a cell sent to N processes counts N times; an
    // unknown neighborhood id gives the maximum uint64_t
    uint64_t get_number_of_update_send_cells(int hood = default_neighborhood_id) const
    {
        if (!hoods_.count(hood)) return std::numeric_limits<uint64_t>::max();
        uint64_t n = 0;
        for (auto& kv : hs(hood).send) n += kv.second.size();
        return n;
    }
    uint64_t get_number_of_update_receive_cells(int hood = default_neighborhood_id) const
    {
        if (!hoods_.count(hood)) return std::numeric_limits<uint64_t>::max();
        uint64_t n = 0;
        for (auto& kv : hs(hood).recv) n += kv.second.size();
        return n;
    }
    // dccrg.hpp:7153-7184: default-constructed copies of the neighborhood's
    // remote neighbors (already present here: build_hood allocates them)
    Dccrg& allocate_copies_of_remote_neighbors(int hood = default_neighborhood_id)
    {
        if (!hoods_.count(hood)) throw std::invalid_argument("Neighborhood with given id doesn't exist.");
        for (uint64_t c : hs(hood).remote_ids) remote_data_[c];
        return *this;
    }
    // dccrg.hpp:2828-2955: face neighbors (the face graph neighbor and, for a
    // smaller one, its siblings sharing the face) with directions +-1/2/3;
    // empty for a cell that is not an existing leaf (the reference aborts)
    std::vector<std::pair<uint64_t, int>> get_face_neighbors_of(uint64_t cell) const
    {
        std::vector<std::pair<uint64_t, int>> out;
        uint64_t row[2] = {0, 0}, ids[24];
        int32_t dirs[24];
        if (dccrgx_face_neighbors_of_host(grid_, &cell, 1, row, ids, dirs, 24) != DCCRGX_OK) return out;
        for (uint64_t e = row[0]; e < row[1]; e++) out.emplace_back(ids[e], (int)dirs[e]);
        return out;
    }
    // dccrg.hpp:3175-3222: the remote neighbors of a local cell (nothing for a
    // cell that is not local or an unknown neighborhood)
    std::vector<uint64_t> get_remote_neighbors_of(uint64_t cell, int hood = default_neighborhood_id,
                                                  bool sorted = false) const
    {
        std::vector<uint64_t> out;
        if (!is_local(cell)) return out;
        const neighbor_list_t* of = get_neighbors_of(cell, hood);
        if (!of) return out;
        for (const auto& x : *of)
            if (x.first != error_cell && get_process(x.first) != rank_) out.push_back(x.first);
        if (sorted) std::sort(out.begin(), out.end());
        return out;
    }
    // dccrg.hpp:3557-3590: every leaf of the grid (the replicated leaf set)
    std::vector<uint64_t> get_all_cells(bool sorted = false) const
    {
        size_t n = 0;
        detail::check(dccrgx_get_all_cells(grid_, nullptr, 0, &n) == DCCRGX_ERANGE || n == 0 ? DCCRGX_OK : DCCRGX_EINVAL,
                      "get_all_cells");
        std::vector<uint64_t> v(n);
        if (n) detail::check(dccrgx_get_all_cells(grid_, v.data(), n, &n), "get_all_cells");
        (void)sorted;  // ascending already
        return v;
    }
    // dccrg.hpp:6840-6858: the default neighborhood's items and their opposites
    std::vector<Types<3>::neighborhood_item_t> get_neighborhood_of() const
    {
        size_t n = 0;
        detail::check(dccrgx_get_neighborhood(grid_, default_neighborhood_id, nullptr, 0, &n) == DCCRGX_ERANGE || n == 0
                          ? DCCRGX_OK
                          : DCCRGX_EINVAL,
                      "get_neighborhood_of");
        std::vector<int32_t> flat(3 * n);
        if (n) detail::check(dccrgx_get_neighborhood(grid_, default_neighborhood_id, flat.data(), n, &n), "items");
        std::vector<Types<3>::neighborhood_item_t> out(n);
        for (size_t i = 0; i < n; i++) out[i] = {{flat[3 * i], flat[3 * i + 1], flat[3 * i + 2]}};
        return out;
    }
    std::vector<Types<3>::neighborhood_item_t> get_neighborhood_to() const
    {
        std::vector<Types<3>::neighborhood_item_t> out = get_neighborhood_of();
        for (auto& it : out) it = {{-it[0], -it[1], -it[2]}};
        return out;
    }
    // dccrg.hpp:6733-6745, 7787-7800: MPI_TAG_UB of the communicator (32767 if unset)
    unsigned int get_max_tag() const
    {
        void* attr = nullptr;
        int flag = 0;
        MPI_Comm_get_attr(comm_, MPI_TAG_UB, &attr, &flag);
        return flag && attr ? (unsigned int)*static_cast<int*>(attr) : 32767u;
    }
    // dccrg.hpp:6836-6842: the local cells' data
    const std::unordered_map<uint64_t, Cell_Data>& get_cell_data() const { return cell_data_; }
    // dccrg.hpp:3225-3287: the remote cells that consider a local cell their
    // neighbor (nothing for a cell that is not local or an unknown neighborhood)
    std::vector<uint64_t> get_remote_neighbors_to(uint64_t cell, int hood = default_neighborhood_id,
                                                  bool sorted = false) const
    {
        std::vector<uint64_t> out;
        if (!is_local(cell)) return out;
        const neighbor_list_t* to = get_neighbors_to(cell, hood);
        if (!to) return out;
        for (const auto& x : *to)
            if (x.first != error_cell && get_process(x.first) != rank_) out.push_back(x.first);
        if (sorted) std::sort(out.begin(), out.end());
        return out;
    }
    std::vector<uint64_t> get_remote_cells_on_process_boundary(int hood = default_neighborhood_id, bool = false) const
    {
        return hoods_.count(hood) ? hs(hood).remote_ids : std::vector<uint64_t>();
    }
    // dccrg.hpp:6953-6975: the owner of every cell of the grid (built from
    // the replicated leaf set on the first call after a structural change,
    // then kept: references stay valid until the next refine / load /
    // neighborhood change) and the default neighborhood's boundary cells as
    // sets.  A uniform grid never replicates cell_process, so a
    // map of more than 2^27 cells is refused rather than built.
    const std::unordered_map<uint64_t, uint64_t>& get_cell_process() const
    {
        if (cp_epoch_ == epoch_) return cell_process_;
        size_t total = 0;
        const int e = dccrgx_get_all_cells(grid_, nullptr, 0, &total);
        detail::check(e == DCCRGX_ERANGE ? DCCRGX_OK : e, "get_all_cells");
        if (total > (uint64_t(1) << 27))
            throw std::length_error("get_cell_process: " + std::to_string(total) +
                                    " cells; the map would be as large as the grid (owners are arithmetic: "
                                    "get_process(cell))");
        const std::vector<uint64_t> all = get_all_cells();
        std::vector<int32_t> owner(all.size());
        if (!all.empty()) detail::check(dccrgx_get_process(grid_, all.data(), all.size(), owner.data()), "get_process");
        cell_process_.clear();
        cell_process_.reserve(all.size());
        for (size_t i = 0; i < all.size(); i++) cell_process_[all[i]] = uint64_t(owner[i]);
        cp_epoch_ = epoch_;
        return cell_process_;
    }
    const std::unordered_set<uint64_t>& get_local_cells_on_process_boundary_internal() const
    {
        if (lb_epoch_ != epoch_) {
            const std::vector<uint64_t> v = get_local_cells_on_process_boundary();
            local_bdy_ = std::unordered_set<uint64_t>(v.begin(), v.end());
            lb_epoch_ = epoch_;
        }
        return local_bdy_;
    }
    const std::unordered_set<uint64_t>& get_remote_cells_on_process_boundary_internal() const
    {
        if (rb_epoch_ != epoch_) {
            const std::vector<uint64_t> v = get_remote_cells_on_process_boundary();
            remote_bdy_ = std::unordered_set<uint64_t>(v.begin(), v.end());
            rb_epoch_ = epoch_;
        }
        return remote_bdy_;
    }
    // the three-phase balance_load (:3745-4150) as built with DCCRG_NO_LB
    // (:3982-4181 compiled out): no cell moves, nothing is added or removed,
    // the caches stay
    Dccrg& initialize_balance_load(bool = true) { return *this; }
    Dccrg& continue_balance_load() { return *this; }
    Dccrg& finish_balance_load() { return *this; }
    const std::unordered_set<uint64_t>& get_cells_added_by_balance_load() const { return no_cells_; }
    const std::unordered_set<uint64_t>& get_cells_removed_by_balance_load() const { return no_cells_; }
    // :3320-3390: an ASCII legacy-VTK unstructured grid of this rank's leaf
    // cells in ascending id order, 8 corner points per cell (x fastest), each
    // cell a voxel (type 11)
    bool write_vtk_file(const std::string& file_name) const
    {
        std::ofstream out(file_name);
        if (!out.is_open()) {
            std::cerr << "Couldn't open file " << file_name << std::endl;
            return false;
        }
        std::vector<uint64_t> leaves = get_cells();
        std::sort(leaves.begin(), leaves.end());
        const size_t n = leaves.size();
        out << "# vtk DataFile Version 2.0\nCartesian cell refinable grid\nASCII\nDATASET UNSTRUCTURED_GRID\n";
        out << "POINTS " << n * 8 << " float\n";
        for (uint64_t c : leaves) {
            const std::array<double, 3> lo = geometry.get_min(c), hi = geometry.get_max(c);
            for (int k = 0; k < 8; k++)
                out << (k & 1 ? hi : lo)[0] << " " << (k & 2 ? hi : lo)[1] << " " << (k & 4 ? hi : lo)[2] << "\n";
        }
        out << "CELLS " << n << " " << n * 9 << "\n";
        for (size_t j = 0; j < n; j++) {
            out << "8 ";
            for (size_t i = 0; i < 8; i++) out << j * 8 + i << " ";
            out << "\n";
        }
        out << "CELL_TYPES " << n << "\n";
        for (size_t i = 0; i < n; i++) out << "11\n";
        return out.good();
    }
    bool get_no_load_balancing() const { return true; }  // :7101-7107, as built with DCCRG_NO_LB
    bool get_balancing_load() const { return false; }    // :7132-7135

    // dccrg.hpp:6491-6711
    bool add_neighborhood(int id, const std::vector<Types<3>::neighborhood_item_t>& items)
    {
        std::vector<int32_t> flat;
        for (const auto& it : items) flat.insert(flat.end(), it.begin(), it.end());
        const int s = dccrgx_add_neighborhood(grid_, id, flat.data(), items.size());
        if (s == DCCRGX_EINVAL) return false;
        detail::check(s, "add_neighborhood");
        build_hood(id);
        user_hood_of_[id] = items;
        auto& to = user_hood_to_[id];
        to.clear();
        for (const auto& it : items) to.push_back({{-it[0], -it[1], -it[2]}});
        return true;
    }
    Dccrg& remove_neighborhood(int id)
    {
        if (id == default_neighborhood_id) return *this;
        detail::check(dccrgx_remove_neighborhood(grid_, id), "remove_neighborhood");
        hoods_.erase(id);
        ++epoch_;
        user_hood_of_.erase(id);
        user_hood_to_.erase(id);
        return *this;
    }
    // dccrg.hpp:6860-6880: the items of the user neighborhoods and their opposites
    const std::unordered_map<int, std::vector<Types<3>::neighborhood_item_t>>& get_user_hood_of() const
    {
        return user_hood_of_;
    }
    const std::unordered_map<int, std::vector<Types<3>::neighborhood_item_t>>& get_user_hood_to() const
    {
        return user_hood_to_;
    }
    // dccrg.hpp:6886-6914: the default neighborhood's lists of every cell here
    const std::unordered_map<uint64_t, neighbor_list_t>& get_all_neighbors_of() const
    {
        return hs(default_neighborhood_id).nof;
    }
    const std::unordered_map<uint64_t, neighbor_list_t>& get_all_neighbors_to() const
    {
        return hs(default_neighborhood_id).nto;
    }
    // dccrg.hpp:6978-7044: per user neighborhood, the cells with a remote
    // neighbor, the remote cells with a local neighbor, and the tagged
    // send / receive lists per process
    const std::unordered_map<int, std::unordered_set<uint64_t>>& get_user_local_cells_on_process_boundary() const
    {
        if (ulb_epoch_ == epoch_) return user_local_bdy_;
        ulb_epoch_ = epoch_;
        user_local_bdy_.clear();
        for (const auto& kv : hoods_)
            if (kv.first != default_neighborhood_id) {
                const std::vector<uint64_t> v = query_cells(kv.first, DCCRGX_CELLS_OUTER);
                user_local_bdy_[kv.first].insert(v.begin(), v.end());
            }
        return user_local_bdy_;
    }
    const std::unordered_map<int, std::unordered_set<uint64_t>>& get_user_remote_cells_on_process_boundary() const
    {
        if (urb_epoch_ == epoch_) return user_remote_bdy_;
        urb_epoch_ = epoch_;
        user_remote_bdy_.clear();
        for (const auto& kv : hoods_)
            if (kv.first != default_neighborhood_id)
                user_remote_bdy_[kv.first].insert(kv.second.remote_ids.begin(), kv.second.remote_ids.end());
        return user_remote_bdy_;
    }
    const std::unordered_map<int, std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>>&
    get_user_neigh_cells_to_send() const
    {
        user_send_.clear();
        for (const auto& kv : hoods_)
            if (kv.first != default_neighborhood_id) user_send_[kv.first] = kv.second.send_tagged;
        return user_send_;
    }
    const std::unordered_map<int, std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>>&
    get_user_neigh_cells_to_receive() const
    {
        user_recv_.clear();
        for (const auto& kv : hoods_)
            if (kv.first != default_neighborhood_id) user_recv_[kv.first] = kv.second.recv_tagged;
        return user_recv_;
    }

    // ---- halo ---------------------------------------------------------------
    // dccrg.hpp:978-1014 (returns false for the default id like the reference,
    // dccrg.hpp:1001-1003, but still transfers)
    bool update_copies_of_remote_neighbors(int hood = default_neighborhood_id)
    {
        if (!start_remote_neighbor_copy_updates(hood)) return false;
        wait_remote_neighbor_copy_updates(hood);
        return hood != default_neighborhood_id;
    }
    // :5046-5078: receives, then sends.  The library moves one update of a
    // neighborhood as one group of RCCL sends and receives (one message per
    // peer, dccrg.hpp:10726-11209), so it is launched once both halves are
    // started (or at the first wait); it then runs on the communication stream
    // while the caller computes, and each wait completes its own half: ghosts
    // are unpacked by wait_..._receives, buffers released by wait_..._sends.
    bool start_remote_neighbor_copy_updates(int hood = default_neighborhood_id)
    {
        if (!start_remote_neighbor_copy_receives(hood)) return false;
        return start_remote_neighbor_copy_sends(hood);
    }
    bool start_remote_neighbor_copy_receives(int hood = default_neighborhood_id)  // :5091-5188
    {
        auto h = hoods_.find(hood);
        if (h == hoods_.end()) return false;
        HoodState& S = h->second;
        if (S.recv_posted) throw std::runtime_error("receives of this neighborhood already started");
        S.rbuf.clear();
        for (auto& kv : S.recv) {
            size_t total = 0;
            for (uint64_t c : kv.second) total += pack_size(c, *(*this)[c], kv.first, rank_, true, hood);
            S.rbuf.emplace_back(total);
        }
        S.recv_posted = true;
        if (S.send_posted) launch(hood, S);
        return true;
    }
    bool start_remote_neighbor_copy_sends(int hood = default_neighborhood_id)  // :5198-5298
    {
        auto h = hoods_.find(hood);
        if (h == hoods_.end()) return false;
        HoodState& S = h->second;
        if (S.send_posted) throw std::runtime_error("sends of this neighborhood already started");
        S.sbuf.clear();
        for (auto& kv : S.send) {
            std::vector<char> buf;
            for (uint64_t c : kv.second) pack(c, *(*this)[c], rank_, kv.first, false, hood, buf);
            S.sbuf.push_back(std::move(buf));
        }
        S.send_posted = true;
        if (S.recv_posted) launch(hood, S);
        return true;
    }
    bool wait_remote_neighbor_copy_updates(int hood = default_neighborhood_id)  // :5307-5338
    {
        if (!hoods_.count(hood)) return false;
        wait_remote_neighbor_copy_update_receives(hood);
        return wait_sends_of(hood, hoods_.at(hood));
    }
    bool wait_remote_neighbor_copy_update_receives(int hood = default_neighborhood_id)  // :5377-5413
    {
        auto h = hoods_.find(hood);
        if (h == hoods_.end()) return false;
        HoodState& S = h->second;
        if (!S.recv_posted) return true;
        complete(hood, S);
        size_t i = 0;
        for (auto& kv : S.recv) {
            int pos = 0;
            for (uint64_t c : kv.second) unpack(c, *(*this)[c], kv.first, rank_, hood, S.rbuf[i], pos);
            i++;
        }
        S.rbuf.clear();
        S.recv_posted = false;
        end_half(S);
        return true;
    }
    // :5347-5368: the sends of every started update
    bool wait_remote_neighbor_copy_update_sends()
    {
        bool ok = true;
        for (auto& kv : hoods_) ok = wait_sends_of(kv.first, kv.second) && ok;
        return ok;
    }
    // :6764-6790: one message per cell instead of one per process.  The bytes
    // each process receives are the same either way and RCCL has no tags, so
    // the mode is recorded (and reported) but moves the same grouped messages.
    Dccrg& set_send_single_cells(const bool given)
    {
        send_single_cells_ = given;
        return *this;
    }
    bool get_send_single_cells() const { return send_single_cells_; }

    // dccrg.hpp:3100-3161: the entries of the cell's neighbors_of whose
    // min-corner indices equal the window at (x, y, z) cell lengths
    // (indices_from_neighborhood, :4236-4352); nothing for a cell that is not
    // local, for (0, 0, 0) or for a window outside a non-periodic grid
    neighbor_list_t get_neighbors_of_at_offset(const uint64_t cell, const int x, const int y, const int z) const
    {
        neighbor_list_t out;
        if (!is_local(cell) || (x == 0 && y == 0 && z == 0)) return out;
        const neighbor_list_t* nof = get_neighbors_of(cell);
        if (!nof) return out;
        const auto idx = mapping.get_indices(cell);
        const uint64_t len = mapping.get_cell_length_in_indices(cell);
        const int off[3] = {x, y, z};
        Types<3>::indices_t ref = idx;
        for (int d = 0; d < 3; d++) {
            const uint64_t glen = mapping.length.get()[d] << mapping.get_maximum_refinement_level();
            if (topology.is_periodic(d)) {  // step by step: the window may wrap several times
                for (int i = 0; i > off[d]; i--) ref[d] = ref[d] >= len ? ref[d] - len : glen - len;
                for (int i = 0; i < off[d]; i++) ref[d] = ref[d] < glen - len ? ref[d] + len : 0;
            } else if (off[d] < 0) {
                if (idx[d] < uint64_t(-off[d]) * len) return out;
                ref[d] -= uint64_t(-off[d]) * len;
            } else {
                if (idx[d] + uint64_t(off[d]) * len >= glen) return out;
                ref[d] += uint64_t(off[d]) * len;
            }
        }
        for (const auto& n : *nof)
            if (mapping.get_indices(n.first) == ref) out.push_back(n);
        return out;
    }

    // device fast path
    dccrgx_grid* device_grid() const { return grid_; }
    dccrgx_ctx* device_context() const { return ctx_; }

private:
    struct HoodState {
        std::vector<Cells_Item> cells;
        std::vector<Neighbors_Item> neighbors;
        Iterator_Storage<Cells_Item> inner, outer, local, remote, all;
        std::unordered_map<uint64_t, neighbor_list_t> nof, nto;
        std::map<int, std::vector<uint64_t>> send, recv;
        std::unordered_map<int, std::vector<std::pair<uint64_t, int>>> send_tagged, recv_tagged;
        std::vector<uint64_t> remote_ids;
        std::vector<std::vector<char>> sbuf, rbuf;
        bool recv_posted = false, send_posted = false;  // started, not yet waited
        bool launched = false, completed = false;        // the grouped transfer
    };

    // the grouped transfer of one update: both halves' buffers (a half the
    // caller has not started yet is started here), then dccrgx_exchange_start
    void launch(int hood, HoodState& S)
    {
        if (S.launched) return;
        if (!S.recv_posted) start_remote_neighbor_copy_receives(hood);
        if (!S.send_posted) start_remote_neighbor_copy_sends(hood);
        if (S.launched) return;  // the line above launched it
        std::vector<const void*> sp;
        std::vector<void*> rp;
        std::vector<uint64_t> sb, rb;
        for (auto& b : S.sbuf) {
            sp.push_back(b.data());
            sb.push_back(b.size());
        }
        for (auto& b : S.rbuf) {
            rp.push_back(b.data());
            rb.push_back(b.size());
        }
        detail::check(dccrgx_exchange_start(grid_, hood, sp.data(), sb.data(), rp.data(), rb.data()),
                      "remote neighbor copy update");
        S.launched = true;
        S.completed = false;
    }
    void complete(int hood, HoodState& S)
    {
        if (!S.launched) launch(hood, S);
        if (!S.completed) {
            detail::check(dccrgx_exchange_wait(grid_, hood), "remote neighbor copy update");
            S.completed = true;
        }
    }
    // after a half is waited: the update is over once both are
    static void end_half(HoodState& S)
    {
        if (!S.recv_posted && !S.send_posted) S.launched = S.completed = false;
    }
    bool wait_sends_of(int hood, HoodState& S)
    {
        if (!S.send_posted) return true;
        complete(hood, S);
        S.sbuf.clear();
        S.send_posted = false;
        end_half(S);
        return true;
    }

    const HoodState& hs(int hood) const
    {
        auto it = hoods_.find(hood);
        if (it == hoods_.end()) throw std::invalid_argument("unknown neighborhood id " + std::to_string(hood));
        return it->second;
    }

    bool request(int (*fn)(dccrgx_grid*, uint64_t, int32_t*), uint64_t cell)
    {
        int32_t r = 0;
        detail::check(fn(grid_, cell, &r), "refinement request");
        return r != 0;
    }

    std::vector<uint64_t> id_list(int (*fn)(const dccrgx_grid*, uint64_t*, size_t, size_t*)) const
    {
        size_t n = 0;
        detail::check(fn(grid_, nullptr, 0, &n), "cell list");
        std::vector<uint64_t> v(n);
        detail::check(fn(grid_, v.data(), n, &n), "cell list");
        return v;
    }

    std::vector<uint64_t> query_cells(int hood, int which) const
    {
        size_t n = 0;
        int s = dccrgx_get_cells(grid_, hood, which, nullptr, 0, &n);
        if (s != DCCRGX_OK && s != DCCRGX_ERANGE) detail::check(s, "get_cells");
        std::vector<uint64_t> v(n);
        detail::check(dccrgx_get_cells(grid_, hood, which, v.data(), n, &n), "get_cells");
        return v;
    }

    std::map<int, std::vector<uint64_t>> peer_lists(int hood, int send) const
    {
        size_t n = 0;
        int s = dccrgx_get_peers(grid_, hood, send, nullptr, nullptr, 0, &n);
        if (s != DCCRGX_OK && s != DCCRGX_ERANGE) detail::check(s, "get_peers");
        std::vector<int32_t> peers(n);
        std::vector<uint64_t> counts(n);
        detail::check(dccrgx_get_peers(grid_, hood, send, peers.data(), counts.data(), n, &n), "get_peers");
        std::map<int, std::vector<uint64_t>> out;
        for (size_t i = 0; i < n; i++) {
            std::vector<uint64_t> ids(counts[i]);
            size_t m = 0;
            detail::check(dccrgx_get_peer_cells(grid_, hood, send, peers[i], ids.data(), ids.size(), &m),
                          "get_peer_cells");
            out[peers[i]] = std::move(ids);
        }
        return out;
    }

    // the iteration cache, dccrg.hpp:11453-11767: inner, outer, remote cells;
    // neighbors per cell as std::set-ordered [only_of][both][only_to]
    void build_hood(int hood)
    {
        ++epoch_;  // the cached sets of the getters below are rebuilt on their next call
        HoodState S;
        const auto inner = query_cells(hood, DCCRGX_CELLS_INNER);
        const auto outer = query_cells(hood, DCCRGX_CELLS_OUTER);
        S.remote_ids = query_cells(hood, DCCRGX_CELLS_REMOTE);
        for (uint64_t c : S.remote_ids) remote_data_[c];  // :7153-7184, constructed in place
        std::vector<uint64_t> order;
        order.insert(order.end(), inner.begin(), inner.end());
        order.insert(order.end(), outer.begin(), outer.end());
        order.insert(order.end(), S.remote_ids.begin(), S.remote_ids.end());
        const size_t n = order.size();
        std::vector<uint64_t> row(n + 1), trow(n + 1);
        detail::check(dccrgx_neighbors_of_host(grid_, hood, order.data(), n, row.data(), nullptr, nullptr, 0),
                      "neighbors_of");
        std::vector<uint64_t> ids(row[n]);
        std::vector<int32_t> off(3 * row[n]);
        detail::check(dccrgx_neighbors_of_host(grid_, hood, order.data(), n, row.data(), ids.data(), off.data(),
                                               ids.size()),
                      "neighbors_of");
        detail::check(dccrgx_neighbors_to_host(grid_, hood, order.data(), n, trow.data(), nullptr, 0),
                      "neighbors_to");
        std::vector<uint64_t> tids(trow[n]);
        detail::check(dccrgx_neighbors_to_host(grid_, hood, order.data(), n, trow.data(), tids.data(), tids.size()),
                      "neighbors_to");
        typedef std::pair<uint64_t, std::array<int, 3>> item;
        std::vector<std::array<size_t, 4>> ranges(n);
        for (size_t i = 0; i < n; i++) {
            neighbor_list_t nof, nto;
            for (uint64_t k = row[i]; k < row[i + 1]; k++)
                nof.push_back({ids[k], {{off[3 * k], off[3 * k + 1], off[3 * k + 2]}}});
            for (uint64_t k = trow[i]; k < trow[i + 1]; k++) nto.push_back({tids[k], {{0, 0, 0}}});
            std::set<item> ids_of(nof.begin(), nof.end()), ids_to(nto.begin(), nto.end());
            std::set<item> only_of, both, only_to = ids_to;
            for (const item& x : ids_of) {
                item t{x.first, {{0, 0, 0}}};
                only_to.erase(t);
                if (ids_to.count(t)) both.insert(x);
                else only_of.insert(x);
            }
            Cells_Item ci{};
            ci.id = order[i];
            ci.data = (*this)[order[i]];
            {  // ACI::update() of every additional cell item, :11548
                int each[] = {0, (ci.ACI::update(*this, ci, ACI()), 0)...};
                (void)each;
            }
            ranges[i][0] = S.neighbors.size();
            for (const auto* group : {&only_of, &both, &only_to})
                for (const item& x : *group) {
                    Neighbors_Item ni{};
                    ni.id = x.first;
                    ni.data = (*this)[x.first];
                    ni.x = x.second[0];
                    ni.y = x.second[1];
                    ni.z = x.second[2];
                    {  // ANI::update() of every additional neighbor item, :11650-11715
                        int each[] = {0, (ni.ANI::update(*this, ci, ni, hood, ANI()), 0)...};
                        (void)each;
                    }
                    S.neighbors.push_back(std::move(ni));
                }
            ranges[i][1] = ranges[i][0] + only_of.size();
            ranges[i][2] = ranges[i][1] + both.size();
            ranges[i][3] = ranges[i][2] + only_to.size();
            S.nof[order[i]] = std::move(nof);
            S.nto[order[i]] = std::move(nto);
            S.cells.push_back(std::move(ci));
        }
        auto b = S.neighbors.cbegin();
        for (size_t i = 0; i < n; i++) {
            S.cells[i].neighbors_of = {b + ranges[i][0], b + ranges[i][2]};
            S.cells[i].neighbors_to = {b + ranges[i][1], b + ranges[i][3]};
            S.cells[i].all_neighbors = {b + ranges[i][0], b + ranges[i][3]};
        }
        auto cb = S.cells.cbegin();
        const size_t ni = inner.size(), no = outer.size();
        S.inner = {cb, cb + ni};
        S.outer = {cb + ni, cb + ni + no};
        S.local = {cb, cb + ni + no};
        S.remote = {cb + ni + no, S.cells.cend()};
        S.all = {cb, S.cells.cend()};
        S.send = peer_lists(hood, 1);
        S.recv = peer_lists(hood, 0);
        for (auto pr : {std::make_pair(&S.send, &S.send_tagged), std::make_pair(&S.recv, &S.recv_tagged)}) {
            for (auto& kv : *pr.first) {
                auto& v = (*pr.second)[kv.first];
                for (size_t i = 0; i < kv.second.size(); i++) v.push_back({kv.second[i], (int)i + 1});
            }
        }
        hoods_[hood] = std::move(S);
    }

    // A cell's bytes are MPI_Pack of its get_mpi_datatype(), as the
    // reference's struct datatypes put them on the wire.  Named (builtin)
    // datatypes -- every caller's cells but variable_neighbour_data's derived
    // structs -- are contiguous: their packed form is the bytes themselves,
    // so they are copied directly with the type's size looked up once.
    // Derived datatypes are flattened into byte blocks (detail::flatten) and
    // copied; only unusual constructors go through MPI_Type_commit / MPI_Pack.
    // The caller's derived type is freed after use, as the reference frees
    // it (dccrg.hpp:10915-10925).
    int named_size(MPI_Datatype t)
    {
        auto it = type_size_.find(t);
        if (it != type_size_.end()) return it->second;
        int sz = 0;
        MPI_Type_size(t, &sz);
        type_size_[t] = sz;
        return sz;
    }
    int pack_size(uint64_t id, Cell_Data& c, int sender, int receiver, bool receiving, int hood)
    {
        auto d = detail::cell_datatype(c, id, sender, receiver, receiving, hood);
        MPI_Datatype t = std::get<2>(d);
        if (detail::is_named(t)) return std::get<1>(d) * named_size(t);
        detail::Blocks fb;
        int sz = 0;
        if (detail::flatten(t, std::get<1>(d), 0, fb)) {
            sz = (int)fb.bytes;
        } else {
            MPI_Type_commit(&t);
            MPI_Pack_size(std::get<1>(d), t, comm_, &sz);
        }
        MPI_Type_free(&t);
        return sz;
    }
    void pack(uint64_t id, Cell_Data& c, int sender, int receiver, bool receiving, int hood, std::vector<char>& buf)
    {
        auto d = detail::cell_datatype(c, id, sender, receiver, receiving, hood);
        MPI_Datatype t = std::get<2>(d);
        if (detail::is_named(t)) {
            const size_t n = (size_t)std::get<1>(d) * named_size(t);
            const size_t at = buf.size();
            buf.resize(at + n);
            if (n) std::memcpy(buf.data() + at, std::get<0>(d), n);
            return;
        }
        detail::Blocks fb;
        if (detail::flatten(t, std::get<1>(d), 0, fb)) {
            size_t at = buf.size();
            buf.resize(at + (size_t)fb.bytes);
            const uintptr_t src = reinterpret_cast<uintptr_t>(std::get<0>(d));  // MPI_BOTTOM + absolute displacements too
            for (const auto& blk : fb.b) {
                std::memcpy(buf.data() + at, reinterpret_cast<const void*>(src + blk.first), (size_t)blk.second);
                at += (size_t)blk.second;
            }
            MPI_Type_free(&t);
            return;
        }
        MPI_Type_commit(&t);
        int sz = 0;
        MPI_Pack_size(std::get<1>(d), t, comm_, &sz);
        int pos = (int)buf.size();
        buf.resize(buf.size() + sz);
        MPI_Pack(std::get<0>(d), std::get<1>(d), t, buf.data(), (int)buf.size(), &pos, comm_);
        buf.resize(pos);
        MPI_Type_free(&t);
    }
    void unpack(uint64_t id, Cell_Data& c, int sender, int receiver, int hood, std::vector<char>& buf, int& pos)
    {
        auto d = detail::cell_datatype(c, id, sender, receiver, true, hood);
        MPI_Datatype t = std::get<2>(d);
        if (detail::is_named(t)) {
            const size_t n = (size_t)std::get<1>(d) * named_size(t);
            if (n) std::memcpy(std::get<0>(d), buf.data() + pos, n);
            pos += (int)n;
            return;
        }
        detail::Blocks fb;
        if (detail::flatten(t, std::get<1>(d), 0, fb)) {
            const uintptr_t dst = reinterpret_cast<uintptr_t>(std::get<0>(d));
            for (const auto& blk : fb.b) {
                std::memcpy(reinterpret_cast<void*>(dst + blk.first), buf.data() + pos, (size_t)blk.second);
                pos += (int)blk.second;
            }
            MPI_Type_free(&t);
            return;
        }
        MPI_Type_commit(&t);
        MPI_Unpack(buf.data(), (int)buf.size(), &pos, std::get<0>(d), std::get<1>(d), t, comm_);
        MPI_Type_free(&t);
    }

    std::unordered_map<uint64_t, Cell_Data> cell_data_, remote_data_, refined_data_, unrefined_data_;
    std::map<int, HoodState> hoods_;
    dccrgx_ctx* ctx_ = nullptr;
    dccrgx_grid* grid_ = nullptr;
    MPI_Comm comm_ = MPI_COMM_NULL;
    int rank_ = 0, size_ = 1;
    uint8_t partition_ = DCCRGX_PARTITION_BLOCK;
    unsigned hood_length_ = 1;
    bool initialized_ = false;
    bool send_single_cells_ = false;
    std::map<MPI_Datatype, int> type_size_;
    std::unordered_map<int, std::vector<Types<3>::neighborhood_item_t>> user_hood_of_, user_hood_to_;
    std::unordered_map<uint64_t, double> cell_weights_;
    // the user-neighborhood views, refreshed by their accessors
    mutable std::unordered_map<int, std::unordered_set<uint64_t>> user_local_bdy_, user_remote_bdy_;
    mutable std::unordered_map<uint64_t, uint64_t> cell_process_;
    uint64_t epoch_ = 0;  // structural changes (build_hood, remove_neighborhood)
    mutable uint64_t cp_epoch_ = ~uint64_t(0), lb_epoch_ = ~uint64_t(0), rb_epoch_ = ~uint64_t(0),
                     ulb_epoch_ = ~uint64_t(0), urb_epoch_ = ~uint64_t(0);
    mutable std::unordered_set<uint64_t> local_bdy_, remote_bdy_;
    const std::unordered_set<uint64_t> no_cells_{};
    mutable std::unordered_map<int, std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>> user_send_,
        user_recv_;
};

}  // namespace dccrg

#endif  // DCCRG_AMD_HPP
