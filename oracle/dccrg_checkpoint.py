"""TEST INFRASTRUCTURE ONLY -- CPU restatement of dccrg's grid data file
(save_grid_data / load_grid_data, dccrg.hpp:1109-2427), the checker for the
device checkpoint path (dccrg_amd/csrc/checkpoint.hip).  Only tests/ and
bench.py's cpu_baseline leg may import this module.

File layout (dccrg.hpp:1124-1142, tests/restart/dc2vtk.cpp:88-98):
  offset bytes skipped; the user's header (rank 0, :1162-1216)
  u64 endianness check 0x1234567890abcdef (:1224-1242)
  mapping: u64 length[3], i32 max_ref_lvl (dccrg_mapping.hpp:615-660)
  u32 neighborhood_length (:1256-1271)
  topology: u8 periodic[3] (dccrg_topology.hpp:170-207)
  geometry: i32 id, then No_Geometry nothing (dccrg_no_geometry.hpp:486-549),
    Cartesian f64 start[3] + f64 level_0_cell_length[3]
    (dccrg_cartesian_geometry.hpp:620-812), Stretched u64 n[3] + f64
    coordinates (dccrg_stretched_cartesian_geometry.hpp:652-817)
  u64 total number of cells (:1286-1310)
  (u64 id, u64 absolute byte offset of its data) per cell, rank by rank, each
    rank's cells in its own order (:1500-1575)
  cell data, rank by rank, same order, each cell the packed bytes of its
    datatype (no padding: contiguous file types, :1385-1420)

Parity note: the reference cannot be built here (Oracle) and ships
no .dc files, so this restatement is pinned by the source above and by the
reference's own reader (dc2vtk.cpp:100-260) -- "parity unpinned" against
reference-written bytes.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Sequence, Tuple

ENDIANNESS = 0x1234567890ABCDEF


def no_geometry() -> bytes:
    return struct.pack("<i", 0)


def cartesian_geometry(start, level_0_cell_length) -> bytes:
    return struct.pack("<i3d3d", 1, *[float(v) for v in start], *[float(v) for v in level_0_cell_length])


def stretched_geometry(coordinates: Sequence[Sequence[float]]) -> bytes:
    out = struct.pack("<i3Q", 2, *[len(c) for c in coordinates])
    for c in coordinates:
        out += struct.pack(f"<{len(c)}d", *[float(v) for v in c])
    return out


def geometry_size(blob_or_file: bytes, at: int = 0) -> int:
    """data_size() of the geometry whose id starts at `at`."""
    (gid,) = struct.unpack_from("<i", blob_or_file, at)
    if gid == 0:
        return 4
    if gid == 1:
        return 4 + 48
    if gid == 2:
        n = struct.unpack_from("<3Q", blob_or_file, at + 4)
        return 4 + 24 + 8 * sum(n)
    raise ValueError(f"unknown geometry id {gid}")


def preamble(length, max_ref_lvl: int, neighborhood_length: int, periodic, geometry: bytes,
             total_cells: int) -> bytes:
    """Everything after the user's header up to the cell list."""
    return (struct.pack("<Q", ENDIANNESS) + struct.pack("<3Qi", *[int(v) for v in length], int(max_ref_lvl))
            + struct.pack("<I", int(neighborhood_length)) + bytes(1 if p else 0 for p in periodic)
            + geometry + struct.pack("<Q", int(total_cells)))


def write_grid_data(offset: int, header: bytes, length, max_ref_lvl: int, neighborhood_length: int,
                    periodic, geometry: bytes,
                    ranks: Sequence[Sequence[Tuple[int, bytes]]], prefix: bytes = b"") -> bytes:
    """The bytes save_grid_data leaves in a file: `ranks` = per rank, its
    cells in writing order as (id, packed data).  `prefix` fills the skipped
    `offset` bytes (save_grid_data does not touch them)."""
    assert len(prefix) == offset
    total = sum(len(r) for r in ranks)
    out = bytearray(prefix + header)
    out += preamble(length, max_ref_lvl, neighborhood_length, periodic, geometry, total)
    list_start = len(out)
    data_start = list_start + 16 * total
    lst = bytearray()
    data = bytearray()
    for r in ranks:
        for cid, payload in r:
            lst += struct.pack("<QQ", int(cid), data_start + len(data))
            data += payload
    return bytes(out + lst + data)


def read_grid_data(buf: bytes, offset: int, header_bytes: int, sizes: Optional[Dict[int, int]] = None) -> Dict:
    """start_loading_grid_data's parse (dccrg.hpp:1815-2072) plus every
    cell's data bytes.  The file does not store record lengths (the reader's
    datatypes give them, :2175-2248): `sizes` maps id -> record bytes;
    without it a record runs to the next record's start (the last to EOF),
    which is right when no record is empty."""
    at = offset
    header = bytes(buf[at:at + header_bytes])
    at += header_bytes
    (endian,) = struct.unpack_from("<Q", buf, at)
    if endian != ENDIANNESS:
        raise ValueError("wrong endianness")
    at += 8
    l0, l1, l2, mrl = struct.unpack_from("<3Qi", buf, at)
    at += 28
    (hood,) = struct.unpack_from("<I", buf, at)
    at += 4
    per = tuple(bool(b) for b in buf[at:at + 3])
    at += 3
    gs = geometry_size(buf, at)
    geometry = bytes(buf[at:at + gs])
    at += gs
    (total,) = struct.unpack_from("<Q", buf, at)
    at += 8
    pairs = [struct.unpack_from("<QQ", buf, at + 16 * i) for i in range(total)]
    starts = sorted(d for _, d in pairs)
    nxt = {d: (starts[k + 1] if k + 1 < len(starts) else len(buf)) for k, d in enumerate(starts)}
    if sizes is None:
        cells = {int(c): bytes(buf[d:nxt[d]]) for c, d in pairs}
    else:
        cells = {int(c): bytes(buf[d:d + sizes[int(c)]]) for c, d in pairs}
    return {"header": header, "length": (l0, l1, l2), "max_ref_lvl": mrl, "neighborhood_length": hood,
            "periodic": per, "geometry": geometry, "total": total, "list_offset": at,
            "order": [int(c) for c, _ in pairs], "offsets": {int(c): int(d) for c, d in pairs}, "cells": cells}
