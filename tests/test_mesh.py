"""Mesh ingest of libpamg (host code, runs on CPU): the O(U) edge-hash
neighbour search must reproduce the reference's O(U^2) CheckNeig topology
exactly (Msh2Tri.F90:776-963, getNeigDataMesh :454-548), pinned against the
reference's own dumps in tests/golden."""
import os

import numpy as np
import pytest

import goldens
import oracle_lib as O
import pamg

MESHES = sorted(f for f in os.listdir(goldens.MESHES) if f.endswith(".msh"))


def golden_for_mesh(mesh):
    for n in goldens.names():
        meta, d = goldens.load(n)
        if meta["mesh"] == mesh:
            return d
    return None


@pytest.mark.parametrize("mesh", MESHES)
def test_topology_equals_reference(mesh):
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))
    d = golden_for_mesh(mesh)
    if d is None:   # no reference dump for this mesh: compare with the pinned oracle
        o = O.read_msh(os.path.join(goldens.MESHES, mesh))
        ref = dict(X=o.X.reshape((2, 3, o.U), order="F"), Neig=o.neig.reshape((3, o.U), order="F"),
                   fNeig=o.fneig.reshape((3, o.U), order="F"), Dir=o.dir.reshape((3, o.U), order="F"),
                   region=np.tile(o.region, (3, 1)))
    else:
        ref = d
    U = m.U
    np.testing.assert_array_equal(m.X.reshape((2, 3, U), order="F"), ref["X"])
    np.testing.assert_array_equal(m.neig.reshape((3, U), order="F"), ref["Neig"])
    np.testing.assert_array_equal(m.fneig.reshape((3, U), order="F"), ref["fNeig"])
    np.testing.assert_array_equal(m.dir.reshape((3, U), order="F"), ref["Dir"])
    np.testing.assert_array_equal(m.region, ref["region"][0])


def test_strip_mesh_topology_is_consistent():
    m = pamg.Mesh.strip(16, 4)
    U = m.U
    assert U == 128
    ne = m.neig.reshape(U, 3)
    fn = m.fneig.reshape(U, 3)
    interior = 0
    for e in range(U):
        for f in range(3):
            n = ne[e, f]
            if n:
                interior += 1
                assert ne[n - 1, fn[e, f] - 1] == e + 1   # symmetric
    # 16x4 cells: interior edges = horizontal 15*4 + vertical 16*3 + diagonals 64
    assert interior == 2 * (15 * 4 + 16 * 3 + 64)


def test_partitions_cover_every_element():
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    for nr in (1, 2, 4, 8):
        for own in (m.x_strip_owner(nr), m.block_owner(nr)):
            counts = np.bincount(own, minlength=nr)
            assert counts.sum() == m.U and counts.min() >= m.U // nr - 1


# ---- synthetic strips, the gmsh writer and the binary mesh cache ----

@pytest.mark.parametrize("nx,ny", [(16, 4), (128, 32)])
def test_strip_written_as_msh_reads_back_through_the_reference_algorithm(tmp_path, nx, ny):
    """pamg_msh_strip's tables are the ones the reference would build from the same triangles:
    the strip written as gmsh 2.2 and read back by ReadMSH + the O(U^2) CheckNeig (the oracle's
    literal restatement, pinned to the reference's own dumps above) and by pamg_msh_read gives
    back X, region, Neig, fNeig and Dir bit for bit."""
    s = pamg.Mesh.strip(nx, ny)
    path = str(tmp_path / "strip.msh")
    s.write_msh(path)
    r = pamg.Mesh.read(path)
    o = O.read_msh(path)
    for m in (r, o):
        assert m.U == s.U
        for k in ("X", "region", "neig", "fneig", "dir"):
            np.testing.assert_array_equal(getattr(m, k), getattr(s, k), err_msg=k)


def test_strip_128x32_has_the_topology_of_untitled8192():
    """untitled8192.msh is gmsh's transfinite mesh of three x-blocks ([0, 0.1] and [0.1, 0.2] at
    dx = 1/320, [0.2, 1] at dx = 1/80) with gmsh's own element order, vertex order (region 11
    clockwise) and coordinate rounding (y = 0.002083333333328173): no generator short of gmsh
    reproduces its X or its local face numbering bit for bit. The synthetic strip 128 x 32
    reproduces its topology: the same element and node counts, the same numbers of interior
    and boundary faces, every interior face shared by exactly two elements."""
    a = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    b = pamg.Mesh.strip(128, 32)

    def stats(m):
        X = m.X.reshape(-1, 3, 2)
        nodes = len({(float(x), float(y)) for x, y in X.reshape(-1, 2)})
        ne = m.neig.reshape(-1, 3)
        fn = m.fneig.reshape(-1, 3)
        for e, f in zip(*np.nonzero(ne)):
            assert ne[ne[e, f] - 1, fn[e, f] - 1] == e + 1
        return m.U, nodes, int((ne > 0).sum()), int((ne == 0).sum())

    assert stats(a) == stats(b) == (8192, 4257, 24256, 320)


def test_binary_mesh_cache_round_trip(tmp_path):
    src = os.path.join(goldens.MESHES, "900_ele.msh")
    msh = str(tmp_path / "m.msh")
    with open(src, "rb") as f, open(msh, "wb") as g:
        g.write(f.read())
    cache = str(tmp_path / "m.pamgmsh")
    ref = pamg.Mesh.read(msh)
    m1, hit1 = pamg.Mesh.read_cached(msh, cache)
    m2, hit2 = pamg.Mesh.read_cached(msh, cache)
    assert (hit1, hit2) == (False, True) and os.path.exists(cache)
    m3 = pamg.Mesh.load(cache)
    for m in (m1, m2, m3):
        for k in ("X", "region", "neig", "fneig", "dir"):
            np.testing.assert_array_equal(getattr(m, k), getattr(ref, k), err_msg=k)
    # a changed .msh invalidates the cache (content hash), a damaged cache is refused and rebuilt
    pamg.Mesh.strip(6, 2).write_msh(msh)
    m4, hit4 = pamg.Mesh.read_cached(msh, cache)
    assert not hit4 and m4.U == 24
    with open(cache, "r+b") as f:
        f.seek(64)
        f.write(b"\xff" * 8)
    with pytest.raises(pamg.PamgError):
        pamg.Mesh.load(cache)
    m5, hit5 = pamg.Mesh.read_cached(msh, cache)
    assert not hit5 and m5.U == 24
