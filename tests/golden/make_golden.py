"""Writes tests/golden/reference_kats.json -- known-answer vectors transcribed
from the reference's own tests (ykempf/dccrg) and from the reference outputs
recorded in SURVEY.md.  Each case names the reference file:line it comes from.

The expected values are written out here with plain index arithmetic for the
tiny grids involved (never computed with the oracle or the product), so that
they pin both independently.  Re-run with ``python tests/golden/make_golden.py``.
"""
import json
import os

E = 0  # dccrg::error_cell


def l1_id(length, x, y, z):
    """Level-1 cell id on a grid of level-0 `length` (max_ref_lvl = 1):
    1 + (#level-0 cells) + x + y*(2Lx) + z*(2Lx)(2Ly)  (dccrg_mapping.hpp:154-209)."""
    n0 = length[0] * length[1] * length[2]
    return 1 + n0 + x + y * 2 * length[0] + z * 4 * length[0] * length[1]


def face_graph_cases():
    """tests/get_neighbors_/test1.cpp -- Dccrg::get_neighbors_() (the face graph,
    order -x,+x,-y,+y,-z,+z), for every neighborhood length 0..3."""
    cases = []
    # 1x1x1, every periodicity (test1.cpp:37-139)
    for per in [(0, 0, 0), (1, 1, 1), (0, 1, 1), (1, 0, 1), (1, 1, 0)]:
        ref = []
        for d in range(3):
            ref += [1, 1] if per[d] else [E, E]
        cases.append({"src": "tests/get_neighbors_/test1.cpp:37-139", "length": [1, 1, 1],
                      "max_ref_lvl": 0, "periodic": per, "refine": [],
                      "expect": {"1": ref}})
    # 3x1x1 / 1x3x1 / 1x1x3, non periodic (test1.cpp:141-265)
    for axis, src in [(0, "141-181"), (1, "183-223"), (2, "225-265")]:
        length = [1, 1, 1]
        length[axis] = 3
        exp = {}
        for c, (lo, hi) in {1: (E, 2), 2: (1, 3), 3: (2, E)}.items():
            r = [E] * 6
            r[2 * axis], r[2 * axis + 1] = lo, hi
            exp[str(c)] = r
        cases.append({"src": f"tests/get_neighbors_/test1.cpp:{src}", "length": length,
                      "max_ref_lvl": 0, "periodic": [0, 0, 0], "refine": [], "expect": exp})
    # 1x1x1 refined once, non periodic and periodic (test1.cpp:268-420)
    L = [1, 1, 1]
    g = lambda x, y, z: l1_id(L, x, y, z)  # noqa: E731
    np_exp, p_exp = {}, {}
    for z in (0, 1):
        for y in (0, 1):
            for x in (0, 1):
                c = g(x, y, z)
                r = [E] * 6
                r[0 if x else 1] = g(1 - x, y, z)
                r[2 if y else 3] = g(x, 1 - y, z)
                r[4 if z else 5] = g(x, y, 1 - z)
                np_exp[str(c)] = r
                o = [g(1 - x, y, z)] * 2 + [g(x, 1 - y, z)] * 2 + [g(x, y, 1 - z)] * 2
                p_exp[str(c)] = o
    cases.append({"src": "tests/get_neighbors_/test1.cpp:268-338", "length": L, "max_ref_lvl": 1,
                  "periodic": [0, 0, 0], "refine": [1], "expect": np_exp})
    cases.append({"src": "tests/get_neighbors_/test1.cpp:340-420", "length": L, "max_ref_lvl": 1,
                  "periodic": [1, 1, 1], "refine": [1], "expect": p_exp})
    # 2x1x1, cell 1 refined (test1.cpp:423-536): get_cell = get_existing_cell(idx, 0, 1)
    L = [2, 1, 1]

    def ex(x, y, z):
        return 2 if x >= 2 else l1_id(L, x, y, z)
    exp = {"2": [ex(1, 0, 0), E, E, E, E, E]}
    for z in (0, 1):
        for y in (0, 1):
            for x in (0, 1):
                r = [E] * 6
                if x == 0:
                    r[1] = ex(1, y, z)
                else:
                    r[0] = ex(0, y, z)
                    r[1] = ex(2, y, z)
                r[2 if y else 3] = ex(x, 1 - y, z)
                r[4 if z else 5] = ex(x, y, 1 - z)
                exp[str(l1_id(L, x, y, z))] = r
    cases.append({"src": "tests/get_neighbors_/test1.cpp:423-536", "length": L, "max_ref_lvl": 1,
                  "periodic": [0, 0, 0], "refine": [1], "expect": exp})
    # 1x2x1, cell 1 refined (test1.cpp:538-626)
    L = [1, 2, 1]

    def ey(x, y, z):
        return 2 if y >= 2 else l1_id(L, x, y, z)
    exp = {"2": [E, E, ey(0, 1, 0), E, E, E]}
    for z in (0, 1):
        for y in (0, 1):
            for x in (0, 1):
                r = [E] * 6
                r[0 if x else 1] = ey(1 - x, y, z)
                if y == 0:
                    r[3] = ey(x, 1, z)
                else:
                    r[2] = ey(x, 0, z)
                    r[3] = ey(x, 2, z)
                r[4 if z else 5] = ey(x, y, 1 - z)
                exp[str(l1_id(L, x, y, z))] = r
    cases.append({"src": "tests/get_neighbors_/test1.cpp:538-626", "length": L, "max_ref_lvl": 1,
                  "periodic": [0, 0, 0], "refine": [1], "expect": exp})
    return cases


def face_neighbor_count_cases():
    """tests/get_face_neighbors/test1.cpp:37-248 -- number of face neighbors
    (get_face_neighbors_of) of every cell."""
    out = []
    for per, n in [((0, 0, 0), 0), ((1, 1, 1), 6), ((0, 1, 1), 4), ((1, 0, 1), 4), ((1, 1, 0), 4)]:
        out.append({"src": "tests/get_face_neighbors/test1.cpp:37-111", "length": [1, 1, 1],
                    "max_ref_lvl": 0, "periodic": per, "refine": [], "count": n})
    for ln in ([2, 1, 1], [1, 2, 1], [1, 1, 2]):
        out.append({"src": "tests/get_face_neighbors/test1.cpp:114-221", "length": ln,
                    "max_ref_lvl": 0, "periodic": [0, 0, 0], "refine": [], "count": 1,
                    "ids": {"1": [2], "2": [1]}})
    out.append({"src": "tests/get_face_neighbors/test1.cpp:224-248", "length": [1, 1, 1],
                "max_ref_lvl": 1, "periodic": [0, 0, 0], "refine": [1], "count": 3})
    return out


def neighbor_list_length_cases():
    """tests/user_neighborhood/neighbor_list_length.cpp:62-310 on a 10^3 fully
    periodic grid with neighborhood length 2: iteration-cache list lengths."""
    hoods = [
        {"id": None, "items": None, "nof": 124, "nto": 124, "src": ":72-91"},
        {"id": 1, "items": [[-2, -2, -2]], "nof": 1, "nto": 1, "src": ":95-125"},
        {"id": 2, "items": [[-2, -2, -2], [2, 2, 2]], "nof": 2, "nto": 2, "src": ":127-160"},
        {"id": -3, "items": [[i, j, 0] for j in range(-2, 3) for i in range(-2, 3)
                            if not (i == 0 and j == 0)], "nof": 24, "nto": 24, "src": ":162-200"},
        {"id": -4, "items": [[0, j, k] for k in range(-2, 3) for j in range(-2, 3)
                            if not (j == 0 and k == 0)], "nof": 24, "nto": 24, "src": ":203-241"},
        {"id": 0, "items": [[i, j, k] for k in range(-2, 3) for j in range(-2, 3)
                            for i in range(-2, 3) if not (i == 0 and j == 0 and k == 0)],
         "nof": 124, "nto": 124, "src": ":244-283"},
    ]
    rejected = [
        {"id": 5, "items": [[-1, 2, -3]], "why": "item beyond neighborhood length", "src": ":286-296"},
        {"id": 0, "items": [[1, 2, -2]], "why": "existing neighborhood id (0 added at :248)", "src": ":298-308"},
    ]
    return {"length": [10, 10, 10], "periodic": [1, 1, 1], "hood_length": 2, "hoods": hoods,
            "rejected": rejected, "src": "tests/user_neighborhood/neighbor_list_length.cpp"}


def gol_kat():
    """tests/game_of_life/game_of_life_test.cpp:54-232 with the initial state of
    tests/game_of_life/initialize.hpp:28-91 (15x15x1 grid, hood 1, not periodic)."""
    gs = 15
    live = set()
    b = 198
    live |= {b, b + 1, b + 2}                                             # blinker
    t = 188
    live |= {t, t + 1, t + 2, t + 1 + gs, t + 2 + gs, t + 3 + gs}          # toad
    be = 137
    live |= {be, be + 1, be - gs, be + 1 - gs, be + 2 - 2 * gs, be + 3 - 2 * gs,
             be + 2 - 3 * gs, be + 3 - 3 * gs}                              # beacon
    gl = 143
    live |= {gl + 1, gl + 2 - gs, gl - 2 * gs, gl + 1 - 2 * gs, gl + 2 - 2 * gs}  # glider
    bl = 47
    live |= {bl, bl + 1, bl - gs, bl + 1 - gs}                              # block
    bh = 51
    live |= {bh - gs, bh + 1, bh + 2, bh + 1 - 2 * gs, bh + 2 - 2 * gs, bh + 3 - gs}  # beehive
    return {
        "src": "tests/game_of_life/game_of_life_test.cpp:54-232, initialize.hpp:28-91",
        "length": [15, 15, 1], "periodic": [0, 0, 0], "hood_length": 1, "steps": 25,
        "initial_live": sorted(live),
        "always_alive": [22, 23, 32, 33, 36, 39, 47, 48, 52, 53, 94, 95, 110, 122, 137, 138,
                         188, 199, 206],
        "alive_even_steps": [109, 123, 189, 190, 198, 200, 204, 205],
        "alive_odd_steps": [174, 184, 214, 220],
        "glider": {"20": [43, 44, 45, 60, 74], "21": [29, 44, 45, 58, 60],
                   "22": [29, 30, 43, 45, 60], "23": [29, 30, 45, 59], "24": [29, 30, 45]},
    }


def simple_gol():
    """examples/simple_game_of_life.cpp:58-158: 10x10x1, hood 1, blinker 54,55,56."""
    return {"src": "examples/simple_game_of_life.cpp:58-158", "length": [10, 10, 1],
            "periodic": [0, 0, 0], "hood_length": 1, "initial_live": [54, 55, 56], "turns": 100,
            "always": [55], "after_even_turn_alive": [45, 65], "after_even_turn_dead": [54, 56],
            "after_odd_turn_alive": [54, 56], "after_odd_turn_dead": [45, 65]}


def line_kat():
    """tests/game_of_life/scalability.cpp:77-213: periodic x,y (z not periodic),
    a line of live cells at y == Ly/2; after k steps exactly the rows
    Ly/2 +- k are alive (k < Ly/2)."""
    return {"src": "tests/game_of_life/scalability.cpp:77-213", "length": [1000, 1000, 1],
            "periodic": [1, 1, 0], "hood_length": 1, "line_y": 500, "steps": 16,
            "alive_rows": [484, 516]}


def survey_facts():
    """Reference outputs recorded during the survey."""
    return [
        {"src": "SURVEY.md 0.3 (dccrg.hpp:7408-7430)", "length": [3, 2, 1], "max_ref_lvl": 0,
         "periodic": [1, 0, 0], "hood_length": 1, "refine": [], "cell": 1, "neighbor": 3,
         "offsets": [[-1, 0, 0]]},
        {"src": "SURVEY.md 0.3", "length": [3, 2, 1], "max_ref_lvl": 1,
         "periodic": [1, 0, 0], "hood_length": 1, "refine": [], "cell": 1, "neighbor": 3,
         "offsets": [[-2, 0, 0]]},
        {"src": "SURVEY.md 0.3 (mixed levels across the wrap)", "length": [4, 1, 1],
         "max_ref_lvl": 1, "periodic": [1, 0, 0], "hood_length": 1, "refine": [1], "cell": 4,
         "neighbor_x_offsets_of_children_of_1": [2, 3]},
        {"src": "SURVEY.md 0.3", "length": [4, 1, 1], "max_ref_lvl": 1, "periodic": [1, 0, 0],
         "hood_length": 1, "refine": [1], "cell": 5, "neighbor": 4,
         "offsets_all_equal": [-2, 0, 0], "min_repeats": 2},
        {"src": "SURVEY.md 0.3 (hood 2 on a 3-cell periodic axis)", "length": [3, 1, 1],
         "max_ref_lvl": 0, "periodic": [1, 0, 0], "hood_length": 2, "refine": [], "cell": 1,
         "axis_sequence": [[2, -2], [3, -1], [2, 1], [3, 2]]},
        {"src": "SURVEY.md 0.4", "length": [3, 3, 1], "max_ref_lvl": 1, "periodic": [0, 0, 0],
         "hood_length": 1, "refine": [5], "cell": 25, "neighbor": 2,
         "offsets": [[-1, -2, 0]] * 4},
    ]


def main():
    out = {
        "face_graph": face_graph_cases(),
        "face_neighbor_counts": face_neighbor_count_cases(),
        "neighbor_list_length": neighbor_list_length_cases(),
        "gol_kat": gol_kat(),
        "simple_gol": simple_gol(),
        "line_kat": line_kat(),
        "survey_facts": survey_facts(),
        "halo_kat": {"src": "examples/basic_cell_data.cpp:27-53", "length": [7, 13, 11],
                     "max_ref_lvl": 1, "hood_length": 2, "periodic": [1, 1, 1],
                     "rule": "after update_copies_of_remote_neighbors every neighbor's data == its id"},
        "mapping_speed_published": {
            "src": "tests/geometry/README:4-24", "length": [100, 200, 300], "max_ref_lvl": 13,
            "ids": "1..1e8", "note": "published timings only (no values), used for the mapping bench"},
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
