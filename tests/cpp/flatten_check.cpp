// The facade's derived-datatype flattening (detail::flatten in
// include/dccrg_amd.hpp) against MPI_Pack / MPI_Unpack: for every constructor
// a cell's get_mpi_datatype may use, the concatenated blocks must be MPI_Pack's
// bytes on this homogeneous run, and copying the bytes back must restore what
// MPI_Unpack restores.  Prints one line per case; exit status 1 on a mismatch.
#include "dccrg_amd.hpp"

#include <cstdio>
#include <functional>
#include <string>
#include <vector>

namespace {

struct Case {
    std::string name;
    std::function<MPI_Datatype(char* base)> make;  // a fresh (uncommitted) type over base
    int count;
};

int check(const Case& c, int& failures)
{
    std::vector<char> mem(4096);
    for (size_t i = 0; i < mem.size(); i++) mem[i] = (char)(i * 37 + 11);
    char* base = mem.data() + 64;
    MPI_Datatype t = c.make(base);
    MPI_Datatype tc = t;
    const bool named = dccrg::detail::is_named(t);
    if (!named) MPI_Type_commit(&tc);
    int sz = 0;
    MPI_Pack_size(c.count, tc, MPI_COMM_SELF, &sz);
    std::vector<char> ref(sz);
    int pos = 0;
    MPI_Pack(base, c.count, tc, ref.data(), sz, &pos, MPI_COMM_SELF);
    ref.resize(pos);
    dccrg::detail::Blocks fb;
    const bool ok = dccrg::detail::flatten(t, c.count, 0, fb);
    std::vector<char> got;
    for (const auto& b : fb.b) got.insert(got.end(), base + b.first, base + b.first + b.second);
    bool same = ok && got == ref;
    // unpack: MPI's and the blocks' into zeroed copies of the memory
    std::vector<char> m1(mem.size(), 0), m2(mem.size(), 0);
    pos = 0;
    MPI_Unpack(ref.data(), (int)ref.size(), &pos, m1.data() + 64, c.count, tc, MPI_COMM_SELF);
    size_t at = 0;
    for (const auto& b : fb.b) {
        std::memcpy(m2.data() + 64 + b.first, got.data() + at, (size_t)b.second);
        at += (size_t)b.second;
    }
    same = same && m1 == m2;
    std::printf("%-28s %s (%zu bytes, %zu blocks)\n", c.name.c_str(), same ? "ok" : "MISMATCH", ref.size(), fb.b.size());
    failures += same ? 0 : 1;
    if (!named) MPI_Type_free(&tc);
    return 0;
}

MPI_Datatype contiguous(MPI_Datatype old, int n)
{
    MPI_Datatype t;
    MPI_Type_contiguous(n, old, &t);
    return t;
}

}  // namespace

int main(int argc, char** argv)
{
    MPI_Init(&argc, &argv);
    int failures = 0;
    std::vector<Case> cases;
    cases.push_back({"named double x3", [](char*) { return MPI_DOUBLE; }, 3});
    cases.push_back({"contiguous int x5", [](char*) { return contiguous(MPI_INT, 5); }, 2});
    cases.push_back({"vector 3x2 stride 5", [](char*) {
                         MPI_Datatype t;
                         MPI_Type_vector(3, 2, 5, MPI_INT, &t);
                         return t;
                     }, 2});
    cases.push_back({"hvector", [](char*) {
                         MPI_Datatype t;
                         MPI_Type_create_hvector(4, 3, 40, MPI_SHORT, &t);
                         return t;
                     }, 1});
    cases.push_back({"indexed", [](char*) {
                         int bl[3] = {2, 1, 3}, dp[3] = {7, 0, 12};
                         MPI_Datatype t;
                         MPI_Type_indexed(3, bl, dp, MPI_DOUBLE, &t);
                         return t;
                     }, 1});
    cases.push_back({"hindexed", [](char*) {
                         int bl[2] = {3, 1};
                         MPI_Aint dp[2] = {100, 8};
                         MPI_Datatype t;
                         MPI_Type_create_hindexed(2, bl, dp, MPI_FLOAT, &t);
                         return t;
                     }, 1});
    cases.push_back({"indexed_block", [](char*) {
                         int dp[3] = {5, 1, 9};
                         MPI_Datatype t;
                         MPI_Type_create_indexed_block(3, 2, dp, MPI_INT, &t);
                         return t;
                     }, 2});
    cases.push_back({"struct with padding", [](char*) {  // {char; double; int[3]} as a C struct lays it out
                         int bl[3] = {1, 1, 3};
                         MPI_Aint dp[3] = {0, 8, 16};
                         MPI_Datatype ty[3] = {MPI_CHAR, MPI_DOUBLE, MPI_INT}, t;
                         MPI_Type_create_struct(3, bl, dp, ty, &t);
                         return t;
                     }, 3});
    cases.push_back({"resized struct", [](char*) {
                         int bl[2] = {1, 1};
                         MPI_Aint dp[2] = {0, 12};
                         MPI_Datatype ty[2] = {MPI_INT, MPI_FLOAT}, s, t;
                         MPI_Type_create_struct(2, bl, dp, ty, &s);
                         MPI_Type_create_resized(s, 0, 32, &t);
                         MPI_Type_free(&s);
                         return t;
                     }, 4});
    cases.push_back({"dup of vector", [](char*) {
                         MPI_Datatype v, t;
                         MPI_Type_vector(2, 1, 3, MPI_LONG, &v);
                         MPI_Type_dup(v, &t);
                         MPI_Type_free(&v);
                         return t;
                     }, 2});
    cases.push_back({"nested struct of vectors", [](char*) {
                         MPI_Datatype v, t;
                         MPI_Type_vector(2, 2, 4, MPI_INT, &v);
                         int bl[2] = {2, 1};
                         MPI_Aint dp[2] = {0, 96};
                         MPI_Datatype ty[2] = {v, MPI_DOUBLE};
                         MPI_Type_create_struct(2, bl, dp, ty, &t);
                         MPI_Type_free(&v);
                         return t;
                     }, 1});
    cases.push_back({"absolute addresses", [](char* base) {  // variable_neighbour_data style: MPI_Get_address
                         MPI_Aint a0, a1, b0;
                         MPI_Get_address(base, &b0);
                         MPI_Get_address(base + 24, &a0);
                         MPI_Get_address(base + 200, &a1);
                         int bl[2] = {1, 5};
                         MPI_Aint dp[2] = {a0 - b0, a1 - b0};
                         MPI_Datatype ty[2] = {MPI_UINT64_T, MPI_DOUBLE}, t;
                         MPI_Type_create_struct(2, bl, dp, ty, &t);
                         return t;
                     }, 1});
    cases.push_back({"double_int pair (gap)", [](char*) { return MPI_DOUBLE_INT; }, 3});
    for (const Case& c : cases) check(c, failures);
    MPI_Finalize();
    return failures ? 1 : 0;
}
