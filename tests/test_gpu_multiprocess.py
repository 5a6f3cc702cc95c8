"""libdccrgx across processes: P ranks as P processes on the one GPU, each
with its own context, exchanging ghosts through the library's host-staged
transport over a gloo process group (tests/mp_worker.py) -- the reference's
transfer engine between distinct ranks (dccrg.hpp:10726-11209), the
collective stop_refining (:3483-3507) and the solvers' cross-rank sums
(tests/poisson/poisson_solve.hpp:349, 426, 486; tests/advection/solve.hpp:317),
checked against the oracle's view of every rank."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SCENARIOS = os.environ.get("MP_SCENARIOS", "gol,gol_explicit,halo_ids,variable,amr,amr_fail,advection,poisson").split(",")
_RESULTS = {}


def run_ranks(P, tmp):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(P):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(P), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        log = open(os.path.join(tmp, f"rank{r}.log"), "w")
        procs.append((subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "mp_worker.py"), tmp,
                                        ",".join(SCENARIOS)], env=env, stdout=log, stderr=subprocess.STDOUT,
                                       start_new_session=True), log))
    rcs = []
    for p, log in procs:
        try:
            rcs.append(p.wait(timeout=600))
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                try:
                    os.killpg(q.pid, 9)
                except OSError:
                    pass
            rcs.append(None)
        log.close()
    out = {}
    for r in range(P):
        f = os.path.join(tmp, f"rank{r}.json")
        out[r] = json.load(open(f)) if os.path.exists(f) else {}
        sys.stdout.write(open(os.path.join(tmp, f"rank{r}.log")).read()[-4000:])
    return rcs, out


@pytest.mark.gpu
@pytest.mark.timeout(1500)
@pytest.mark.parametrize("P", [2, 3, 8])  # 8: configs[4]'s "across 8 MI355X" shapes (8 seams, 8-way sums)
@pytest.mark.parametrize("scenario", SCENARIOS)
def test_multiprocess(P, scenario, tmp_path_factory):
    if P not in _RESULTS:
        _RESULTS[P] = run_ranks(P, str(tmp_path_factory.mktemp(f"mp{P}")))
    rcs, out = _RESULTS[P]
    for r in range(P):
        got = out[r].get(scenario, f"rank {r} wrote no result (exit {rcs[r]})")
        assert got == "ok", f"rank {r}: {got}"
