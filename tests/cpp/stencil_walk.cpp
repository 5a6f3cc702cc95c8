// Host run of include/dccrgx_stencil.hpp's uniform neighbor walk (the same
// code the device functors run), for the CPU test of its iteration order
// (tests/test_user_stencil_walk.py).  The item table is made as stencil.hip
// build_iter makes it.
// stdin: LA LB LC pa pb pc lo hi cbase K, then K canonical items (a b c)
// stdout per local cell: id n, then n x (neighbor id, x, y, z)
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dccrgx_stencil.hpp"

int main()
{
    long long LA, LB, LC, lo, hi, cbase;
    int pa, pb, pc, K;
    if (std::scanf("%lld %lld %lld %d %d %d %lld %lld %lld %d", &LA, &LB, &LC, &pa, &pb, &pc, &lo, &hi, &cbase, &K) != 10)
        return 2;
    std::vector<std::array<int32_t, 4>> it(K);
    int32_t reach[3] = {0, 0, 0};
    for (int k = 0; k < K; k++) {
        if (std::scanf("%d %d %d", &it[k][0], &it[k][1], &it[k][2]) != 3) return 2;
        for (int a = 0; a < 3; a++) reach[a] = std::max(reach[a], std::abs(it[k][a]));
    }
    for (int k = 0; k < K; k++) {
        bool mirror = false;
        for (int j = 0; j < K && !mirror; j++)
            mirror = it[j][0] == -it[k][0] && it[j][1] == -it[k][1] && it[j][2] == -it[k][2];
        it[k][3] = mirror ? 1 : 0;
    }
    std::sort(it.begin(), it.end(), [](const std::array<int32_t, 4>& x, const std::array<int32_t, 4>& y) {
        if (x[3] != y[3]) return x[3] < y[3];
        if (x[2] != y[2]) return x[2] < y[2];
        if (x[1] != y[1]) return x[1] < y[1];
        return x[0] < y[0];
    });
    const long long S = LA * LB;
    std::vector<int32_t> rec(std::max(K, 1) * 8, 0);
    std::vector<int64_t> delta(std::max(K, 1), 0);
    for (int k = 0; k < K; k++) {  // identity axis order, scale 1
        const int32_t r[8] = {it[k][0], it[k][1], it[k][2], it[k][3], it[k][0], it[k][1], it[k][2], 0};
        std::copy(r, r + 8, &rec[8 * k]);
        delta[k] = it[k][0] + LA * it[k][1] + S * it[k][2];
    }
    dccrgx_user::detail::UniformGeo g{};
    g.la = LA, g.lb = LB, g.lc = LC, g.S = S, g.lo = lo, g.hi = hi, g.cbase = cbase;
    g.items = rec.data(), g.delta = delta.data(), g.K = K;
    g.pa = pa, g.pb = pb, g.pc = pc, g.ra = reach[0], g.rb = reach[1], g.rc = reach[2];
    for (long long lin = lo; lin < hi; lin++) {
        dccrgx_user::UniformCell cell;
        cell.g = g;
        cell.c = lin / S;
        cell.b = (lin - cell.c * S) / LA;
        cell.a = lin - cell.c * S - cell.b * LA;
        cell.slot = lin - cbase * S;
        cell.id = lin + 1;
        std::vector<std::array<long long, 4>> out;
        cell.for_each_neighbor([&](const dccrgx_user::Neighbor& nb) {
            // slot -> id: storage slice (unwrapped c) back to the grid
            const long long s = (long long)nb.slot, cs = s / S + cbase, rem = s % S;
            const long long cw = ((cs % LC) + LC) % LC;
            out.push_back({rem + cw * S + 1, nb.x, nb.y, nb.z});
        });
        std::printf("%lld %zu", lin + 1, out.size());
        for (auto& e : out) std::printf(" %lld %lld %lld %lld", e[0], e[1], e[2], e[3]);
        std::printf("\n");
    }
    return 0;
}
