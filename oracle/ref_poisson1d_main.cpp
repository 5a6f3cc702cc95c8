/* TEST INFRASTRUCTURE ONLY.  The reference's serial 1-D Poisson solver
 * (tests/poisson/reference_poisson_solve.hpp, Hockney & Eastwood, compiled
 * where it lies) on poisson1d.cpp's problem (:153-162): n cells over
 * [0, 2 pi], rhs = sin((i + 0.5) dx).  Writes the n solution values (f64) to
 * stdout.  Built by `make -C oracle ref` into oracle/_ref/;
 * tests/test_gpu_ref_poisson.py holds the device BiCG solver to it with
 * poisson1d.cpp's own criterion.  argv: n */
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "reference_poisson_solve.hpp"

int main(int argc, char** argv)
{
    if (argc != 2) return 1;
    const size_t n = std::strtoull(argv[1], nullptr, 10);
    const double dx = 2 * M_PI / n;
    Reference_Poisson_Solve solver(n, dx);
    for (size_t i = 0; i < n; i++) solver.get_rhs(i) = std::sin((i + 0.5) * dx);
    solver.solve();
    for (size_t i = 0; i < n; i++) {
        const double v = solver.get_solution(i);
        std::fwrite(&v, 8, 1, stdout);
    }
    return 0;
}
