// FlatSet / FlatMap32 (dccrg_amd/csrc/flatset.hpp) against std::set / std::map
// under random inserts, erases and lookups, including ids that collide in
// the table.
#include <cstdio>
#include <random>
#include <map>
#include <set>

#include "flatset.hpp"

int main()
{
    std::mt19937_64 rng(7);
    for (int round = 0; round < 40; round++) {
        dccrgx::FlatSet f;
        std::set<uint64_t> s;
        const uint64_t range = round % 2 ? 64 : 1 + (rng() % 100000);
        for (int op = 0; op < 20000; op++) {
            const uint64_t x = rng() % (range + 1);  // 0 (error_cell) is never stored
            switch (rng() % 4) {
            case 0:
            case 1: {
                const bool a = f.insert(x).second, b = x && s.insert(x).second;
                if (a != b) return std::printf("insert %llu\n", (unsigned long long)x), 1;
                break;
            }
            case 2:
                if (f.erase(x) != s.erase(x)) return std::printf("erase %llu\n", (unsigned long long)x), 1;
                break;
            default:
                if (f.count(x) != s.count(x)) return std::printf("count %llu\n", (unsigned long long)x), 1;
            }
            if (f.size() != s.size()) return std::printf("size\n"), 1;
        }
        const std::vector<uint64_t> v = f.sorted();
        if (v != std::vector<uint64_t>(s.begin(), s.end())) return std::printf("sorted\n"), 1;
        size_t n = 0;
        for (uint64_t x : f) n += s.count(x);
        if (n != s.size()) return std::printf("iteration\n"), 1;
        f.clear();
        if (!f.empty() || f.count(v.empty() ? 1 : v[0])) return std::printf("clear\n"), 1;
    }
    for (int round = 0; round < 40; round++) {
        dccrgx::FlatMap32 f;
        std::map<uint64_t, uint32_t> m;
        const uint64_t range = round % 2 ? 64 : 1 + (rng() % 100000);
        for (int op = 0; op < 20000; op++) {
            const uint64_t x = 1 + rng() % range;
            switch (rng() % 3) {
            case 0: {
                const uint32_t v = (uint32_t)rng();
                f.set(x, v);
                m[x] = v;
                break;
            }
            case 1:
                if (f.erase(x) != m.erase(x)) return std::printf("map erase %llu\n", (unsigned long long)x), 1;
                break;
            default: {
                const uint32_t* p = f.find(x);
                auto it = m.find(x);
                if ((p == nullptr) != (it == m.end()) || (p && *p != it->second))
                    return std::printf("map find %llu\n", (unsigned long long)x), 1;
            }
            }
            if (f.size() != m.size()) return std::printf("map size\n"), 1;
        }
    }
    for (size_t n : {0, 5, 4095, 4096, 100000, 100001}) {  // radix_sort_u64 against std::sort
        std::vector<uint64_t> v(n);
        for (auto& x : v) x = (n % 2 ? rng() : (rng() % 1000003) * 8 + 1);
        std::vector<uint64_t> w = v;
        dccrgx::radix_sort_u64(v);
        std::sort(w.begin(), w.end());
        if (v != w) return std::printf("radix sort %zu\n", n), 1;
    }
    std::printf("PASS\n");
    return 0;
}
