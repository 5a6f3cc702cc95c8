import sys
sys.path.insert(0, '.')
import numpy as np
import dccrg_amd as D
from dccrg_amd import advection as A
from oracle.dccrg_amr import AdvectionAmrOracle, AmrOracle
ctx = D.Context(0, 0, 1)
g = (D.Dccrg().set_initial_length((16, 16, 1)).set_maximum_refinement_level(2)
     .set_periodic(True, True, False).set_neighborhood_length(0).initialize(ctx))
g.add_advection_fields()
geom = A.CartesianGeometry(g)
A.initialize(g, geom)
ref = AdvectionAmrOracle.__new__(AdvectionAmrOracle)
ref.o = AmrOracle((16, 16, 1), 2, (True, True, False), 0, 1)
ref.l0 = np.array([1.0 / 16] * 3); ref.params = (0.025, 0.25, 0.5); ref.cfl = 0.5
ref._init_state()
for it in range(2):
    sets = A.check_for_adaptation(g, 0.0125, 0.25, 0.5)
    rs = ref.check_for_adaptation()[0]
    for k in range(3):
        a, b = [int(c) for c in sets[k]], rs[k]
        print(it, k, len(a), len(b), a == b, sorted(set(a) ^ set(b))[:10])
    A.adapt_grid(g, geom, *sets)
    ref.adapt([rs])
    A.initialize(g, geom); ref._init_state()
    gc = [int(c) for c in g.local_cells()]
    print("leaves", len(gc), len(ref.o.cells()), gc == ref.o.cells(), sorted(set(gc) ^ set(ref.o.cells()))[:10])
    rc, ra = ref.arrays()
    if gc == rc:
        print("rho diff", np.max(np.abs(g.read_local("density") - ra[0])))
    if gc == rc:
        d = g.read_local("density")
        bad = np.nonzero(np.abs(d - ra[0]) > 1e-12)[0][:8]
        m = g.mapping
        for i in bad:
            c = gc[i]
            print(c, m.get_refinement_level(c), m.get_indices(c), d[i], ra[0][i], ref._geom(c)[0],
                  geom.centers_and_lengths(np.array([c], dtype=np.uint64))[0])
