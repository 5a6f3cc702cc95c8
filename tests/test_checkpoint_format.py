"""Grid data file layout (save_grid_data / load_grid_data, dccrg.hpp:1109-2427)
on the CPU: the oracle's restatement round-trips, and the library's
host-side parser (dccrgx_file_read_info, no GPU involved) reads the
oracle-written preamble for every geometry kind, header size and offset."""
import os
import struct

import numpy as np
import pytest

import dccrg_amd as D
from oracle import dccrg_checkpoint as K

GEOMS = [K.no_geometry(), K.cartesian_geometry((0.5, -1.0, 2.0), (0.25, 0.125, 1.0)),
         K.stretched_geometry([[0.0, 1.0, 3.0], [0.0, 2.0], [-1.0, 0.0, 0.5, 4.0]])]


def sample(seed=0):
    rng = np.random.default_rng(seed)
    ranks = []
    nxt = 1
    for r in range(3):
        cells = []
        for _ in range(int(rng.integers(0, 5))):
            cells.append((nxt, bytes(rng.integers(0, 256, int(rng.integers(0, 9)), dtype=np.uint8))))
            nxt += int(rng.integers(1, 4))
        ranks.append(cells)
    if not any(ranks):
        ranks[0].append((1, b"x"))
    return ranks


@pytest.mark.parametrize("geom", range(len(GEOMS)))
@pytest.mark.parametrize("offset,header", [(0, b""), (16, b"hdr"), (3, struct.pack("<Q", 25))])
def test_oracle_round_trip(geom, offset, header):
    ranks = sample(geom)
    buf = K.write_grid_data(offset, header, (7, 5, 3), 2, 1, (True, False, True), GEOMS[geom], ranks,
                            prefix=b"\0" * offset)
    flat = [c for r in ranks for c in r]
    got = K.read_grid_data(buf, offset, len(header), sizes={c: len(b) for c, b in flat})
    assert got["header"] == header and got["length"] == (7, 5, 3) and got["max_ref_lvl"] == 2
    assert got["neighborhood_length"] == 1 and got["periodic"] == (True, False, True)
    assert got["geometry"] == GEOMS[geom]
    assert got["order"] == [c for c, _ in flat]
    assert got["cells"] == dict(flat)
    # the list is followed immediately by rank 0's first record (:1500-1507)
    assert got["list_offset"] + 16 * len(flat) == min(got["offsets"].values())


@pytest.mark.parametrize("geom", range(len(GEOMS)))
@pytest.mark.parametrize("offset,header", [(0, b""), (16, b"hdr"), (5, b"\x01" * 11)])
def test_library_parses_oracle_preamble(tmp_path, geom, offset, header):
    ranks = sample(geom + 7)
    buf = K.write_grid_data(offset, header, (9, 4, 2), 3, 2, (False, True, True), GEOMS[geom], ranks,
                            prefix=b"\xee" * offset)
    path = str(tmp_path / "g.dc")
    open(path, "wb").write(buf)
    info, hdr, geo = D.Dccrg.read_file_info(path, offset, len(header))
    ref = K.read_grid_data(buf, offset, len(header))
    assert hdr == header and geo == GEOMS[geom]
    assert tuple(info.params.length) == (9, 4, 2) and info.params.max_ref_lvl == 3
    assert info.params.neighborhood_length == 2 and tuple(info.params.periodic) == (0, 1, 1)
    assert info.geometry_bytes == len(GEOMS[geom]) == K.geometry_size(geo)
    assert info.total_cells == ref["total"] and info.list_offset == ref["list_offset"]
    assert D.lib().dccrgx_file_preamble_bytes(len(GEOMS[geom])) == len(K.preamble((1, 1, 1), 0, 0, (0, 0, 0),
                                                                                 GEOMS[geom], 0))


def test_library_rejects_wrong_endianness(tmp_path):
    buf = bytearray(K.write_grid_data(0, b"", (2, 2, 2), 0, 1, (0, 0, 0), K.no_geometry(), [[(1, b"a")]]))
    buf[0:8] = struct.pack(">Q", K.ENDIANNESS)
    path = str(tmp_path / "bad.dc")
    open(path, "wb").write(bytes(buf))
    with pytest.raises(D.DccrgxError, match="endianness"):
        D.Dccrg.read_file_info(path)
    with pytest.raises(D.DccrgxError):
        D.Dccrg.read_file_info(os.path.join(str(tmp_path), "missing.dc"))
