"""The face-coupled operator (pamg_params.op = 1).

The reference leaves its surface terms commented out and cannot run them (Mesh%S_nodes is never
allocated), so there is no reference output: the operator is defined by the oracle's restatement
(oracle/pamg_oracle.c face_setup / face_terms / face_sweep) and the HIP path is held to it bit
for bit (the oracle takes the device's source term s', as in tests/test_contracted_oracle.py).
CPU tests: the restatement is a well-posed operator for multigrid -- the corrected V-cycle
contracts the level-1 residual cycle after cycle -- and it really couples elements.
GPU tests: every field of every level and t_overlap equal the oracle's, single domain and on
partitions, where the halo is now read every sweep (exchanged through the multi-rank path)."""
import os

import numpy as np
import pytest

import goldens
import oracle_lib as O


def oracle(mesh, S, L, **kw):
    return O.Oracle(O.read_msh(os.path.join(goldens.MESHES, mesh)), S, L, op=1, **kw)


@pytest.mark.parametrize("mesh,S,L,rate", [("untitled8.msh", 3, 3, 0.3), ("irregular.msh", 3, 3, 0.3),
                                           ("900_ele.msh", 3, 3, 0.3), ("test_sn2.msh", 4, 3, 0.5)])
@pytest.mark.parametrize("solver", [1, 3])
def test_corrected_cycle_converges_with_the_face_operator(mesh, S, L, rate, solver):
    o = oracle(mesh, S, L, solver=solver, ntime=1, n_multigrid=1)
    o.begin_timestep()
    r = []
    for _ in range(8):
        o.vcycle_corrected()
        r.append(float(np.abs(o.get(O.RES, 1)).max()))
    assert all(np.isfinite(r))
    assert r[-1] < r[0] * rate ** 6, r
    assert r[-1] < r[-2] < r[-3], r


def test_face_coupling_is_not_block_diagonal():
    """A sweep of op = 1 differs from op = 0 only through the face terms: with a random iterate
    the two differ, and they agree again when the neighbours are frozen at the sub-element's own
    values and k = 0 (no diffusion, no penalty)."""
    rng = np.random.default_rng(20251015)
    a = oracle("untitled8.msh", 2, 1, ntime=1, n_multigrid=1)
    b = O.Oracle(O.read_msh(os.path.join(goldens.MESHES, "untitled8.msh")), 2, 1, ntime=1, n_multigrid=1)
    x = rng.uniform(-1, 1, (3, a.nsub(1), 8))
    for o in (a, b):
        o.set(O.TNEW, 1, x)
        o.begin_timestep()
        o.copy_to_tnn(1)
        o.smoother(1)
    assert np.abs(a.get(O.TNN, 1) - b.get(O.TNN, 1)).max() > 1e-6
    a0 = oracle("untitled8.msh", 2, 1, ntime=1, n_multigrid=1, k=0.0)
    b0 = O.Oracle(O.read_msh(os.path.join(goldens.MESHES, "untitled8.msh")), 2, 1, ntime=1, n_multigrid=1, k=0.0)
    for o in (a0, b0):
        o.set(O.TNEW, 1, x)
        o.begin_timestep()
        o.copy_to_tnn(1)
        o.smoother(1)
    np.testing.assert_array_equal(a0.get(O.TNN, 1), b0.get(O.TNN, 1))


def test_face_operator_rejects_unsupported_configs():
    m = O.read_msh(os.path.join(goldens.MESHES, "untitled8.msh"))
    for kw in (dict(solver=2), dict(coarse_solver=1)):
        with pytest.raises(ValueError):
            O.Oracle(m, 2, 2, op=1, **kw)


# ---------------------------------------------------------------- GPU parity
def gpu_pair(mesh, S, L, solver=3, cycle=0, ns=4):
    import pamg
    path = os.path.join(goldens.MESHES, mesh)
    g = pamg.SemiImplicitIterative(pamg.Mesh.read(path), S, L, n_smooth=ns, solver=solver, cycle=cycle, op=1)
    o = oracle(mesh, S, L, n_smooth=ns, solver=solver)
    o.set_source(g.get(pamg.SOURCE, 1))
    return g, o


def drive(s, is_oracle, cycle, steps=2, cycles=2):
    for _ in range(steps):
        s.begin_timestep()
        for _ in range(cycles):
            if is_oracle:
                s.vcycle_corrected() if cycle else s.vcycle()
        if not is_oracle:
            s.vcycle(cycles)


def assert_identical(sg, so):
    for k in so:
        np.testing.assert_array_equal(sg[k], so[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,solver,ns", [
    ("untitled8.msh", 3, 3, 3, 4), ("untitled8.msh", 3, 3, 1, 2), ("irregular.msh", 4, 3, 3, 2),
    ("900_ele.msh", 3, 2, 3, 3), ("test_sn2.msh", 4, 2, 1, 1), ("untitled8192.msh", 3, 3, 3, 4),
    # the fused single-domain sweep's tiles of 1,024 and 4,096 sub-elements
    ("irregular.msh", 5, 3, 3, 2), ("irregular.msh", 6, 2, 3, 1), ("irregular.msh", 6, 2, 1, 1),
    # one sweep per call (every sweep of the fused cycle's non-final calls is dead), one level
    ("irregular.msh", 4, 3, 3, 1), ("untitled8.msh", 3, 1, 3, 2),
    # bench.py's extra.op1 configuration (untitled8192, n_split 5, L 3, n_smooth 4, solver 3): level 3
    # (64 sub-elements per un_ele, m = 8 face positions) runs as the persistent chain -- 256 cooperating
    # workgroups handing the halo words over inside the launch, the split up pass and the 16-byte
    # write-through snapshot loads (buffer_load_dwordx4 sc1) -- and Jacobi on the same chain
    ("untitled8192.msh", 5, 3, 3, 4), ("untitled8192.msh", 5, 3, 1, 4)])
@pytest.mark.parametrize("cycle", [0, 1])
def test_face_operator_is_bitwise_the_oracle(mesh, S, L, solver, ns, cycle):
    g, o = gpu_pair(mesh, S, L, solver, cycle, ns)
    drive(g, False, cycle)
    drive(o, True, cycle)
    sg, so = g.state(), o.state()
    sg["t_overlap"], sg["t_overlap_old"] = g.overlap()
    so["t_overlap"], so["t_overlap_old"] = o.overlap()
    assert_identical(sg, so)


@pytest.mark.gpu
@pytest.mark.parametrize("solver", [3, 1])
def test_face_chain_8byte_snapshot_is_bitwise_the_oracle(solver, monkeypatch):
    """The chain's snapshot falls back to 8-byte write-through loads when the snapshot buffer exceeds a
    buffer resource's 32-bit range (pamg_face.hip k_face_chain, snap16); PAMG_CHAIN_SNAP16=0 forces that
    form on bench.py's extra.op1 configuration, which must stay bitwise the oracle."""
    monkeypatch.setenv("PAMG_CHAIN_SNAP16", "0")
    g, o = gpu_pair("untitled8192.msh", 5, 3, solver, 0, 4)
    drive(g, False, 0)
    drive(o, True, 0)
    sg, so = g.state(), o.state()
    sg["t_overlap"], sg["t_overlap_old"] = g.overlap()
    so["t_overlap"], so["t_overlap_old"] = o.overlap()
    assert_identical(sg, so)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,parts,kind,solver,cycle,agg", [
    ("untitled8192.msh", 3, 3, 4, "strip", 3, 0, "1"), ("untitled8192.msh", 3, 2, 8, "strip", 3, 1, "1"),
    ("irregular.msh", 4, 2, 8, "strip", 1, 1, "1"), ("900_ele.msh", 2, 2, 3, "block", 3, 0, "1"),
    ("untitled8192.msh", 4, 3, 8, "block", 1, 0, "1"),
    # bench.py's op=1 configuration (n_split 5, L 3, GS) on 8 x-strips and 4 blocks, both cycles: levels of
    # 1,024 / 256 sub-elements per un_ele as one tile launch per sweep, each launch's next-sweep words exchanged
    # into the snapshot buffer that sweep reads; level 3 agglomerated (the ranks' RHS gathered each cycle into a
    # replica of the whole level, the single-domain chain on every rank)
    ("untitled8192.msh", 5, 3, 8, "strip", 3, 0, "1"), ("untitled8192.msh", 5, 3, 8, "strip", 3, 1, "1"),
    ("untitled8192.msh", 5, 3, 4, "block", 3, 0, "1"), ("untitled8192.msh", 5, 3, 4, "block", 3, 1, "1"),
    # PAMG_FACE_AGG=0: the coarsest level partitioned too, one launch and one exchange per sweep
    ("untitled8192.msh", 5, 3, 4, "strip", 3, 0, "0"), ("irregular.msh", 4, 2, 8, "strip", 1, 1, "0"),
    # four levels: two partitioned levels below the agglomerated one
    ("900_ele.msh", 4, 4, 4, "strip", 3, 0, "1"), ("untitled8192.msh", 4, 4, 8, "block", 1, 1, "1"),
    ("test_sn2.msh", 4, 4, 3, "strip", 3, 1, "1")])
def test_face_operator_partitions_match_single_domain(mesh, S, L, parts, kind, solver, cycle, agg, monkeypatch):
    """The halo is consumed every sweep: the partitions' exchanges (the multi-rank path with the
    device-copy transport, tests/test_multirank.py) carry the values the sweeps read -- after every
    launch that writes a sweep's words, into the snapshot buffer the next sweep reads. The coarsest level is
    agglomerated: per cycle one gather of its RHS and at most two coarsest-level launches
    (the chain), instead of a launch and an exchange per sweep."""
    import pamg
    from pamg.solver import local_group, run_ranks
    monkeypatch.setenv("PAMG_FACE_AGG", agg)
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))
    full = pamg.SemiImplicitIterative(m, S, L, solver=solver, cycle=cycle, op=1)
    drive(full, False, cycle)
    owner = m.x_strip_owner(parts) if kind == "strip" else m.block_owner(parts)
    ps = [pamg.SemiImplicitIterative(m, S, L, solver=solver, cycle=cycle, op=1, comm=(parts, r, None, owner))
          for r in range(parts)]
    local_group(ps)
    for p in ps:
        p.timing_enable(1 << 6 | 1 << 17)   # PAMG_K_HALO, PAMG_K_COARSE_GATHER
        p.timing_reset()
    steps, cycles, ns = 2, 2, 4
    run_ranks(ps, lambda p: drive(p, False, cycle, steps, cycles))
    ref, ref_ov = full.state(), full.overlap()
    for r, p in enumerate(ps):
        own = np.flatnonzero(owner == r)
        for k, v in p.state().items():
            np.testing.assert_array_equal(v, ref[k][:, :, own], err_msg=f"rank {r} {k}")
        for x, y in zip(p.overlap(), ref_ov):
            np.testing.assert_array_equal(x, y[:, :, own])
        tm = p.timing()
        n_cycles = steps * cycles
        if agg == "1":
            # the RHS every cycle, tnew once per call (the reference cycle) -- the corrected one starts from zero
            assert tm["coarse_gather"]["issued"] == n_cycles + (0 if cycle else steps), tm["coarse_gather"]
            # exchanges only around the sweeps of levels 1 .. L-1 (their two calls' sweeps and the residuals' refreshes):
            # the coarsest level's 62 sweeps exchange nothing (in a local group its replica runs them one launch per
            # sweep, the ranks sharing one GPU; one process per GPU runs them as the chain: test_rccl_self.py)
            assert tm["halo"]["issued"] <= (L - 1) * (2 * ns + 2) * n_cycles, tm["halo"]
        else:
            assert tm["coarse_gather"]["issued"] == 0
        p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,solver,ns", [("untitled8192.msh", 4, 3, 3, 4), ("irregular.msh", 6, 3, 1, 2),
                                                ("900_ele.msh", 3, 3, 3, 1), ("test_sn2.msh", 4, 4, 3, 3)])
def test_face_fused_cycle_equals_per_step_sequence(mesh, S, L, solver, ns):
    """The fused face V-cycle (vcycle_face_fused: dead last sweeps and the dead prolongator dropped,
    the residual reading the halo its smoother call left) leaves the per-step sequence's state bit
    for bit, whatever the split of the cycles into calls (only a call's last cycle runs its calls'
    last sweeps)."""
    import pamg
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))
    ref = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=solver, op=1, fused=0)
    ref.begin_timestep()
    ref.vcycle(4)
    rs, rov = ref.state(), ref.overlap()
    for split in ([4], [1, 3], [1, 1, 1, 1]):
        g = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=solver, op=1)
        g.begin_timestep()
        for n in split:
            g.vcycle(n)
        assert_identical(g.state(), rs)
        for x, y in zip(g.overlap(), rov):
            np.testing.assert_array_equal(x, y)
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,solver,ns,n", [
    ("untitled8192.msh", 5, 3, 3, 4, 2), ("untitled8192.msh", 5, 2, 1, 3, 1), ("untitled8192.msh", 4, 3, 3, 4, 2),
    ("900_ele.msh", 5, 3, 3, 4, 2), ("irregular.msh", 6, 2, 3, 3, 1)])
def test_face_wavefront_call_equals_per_sweep_launches(mesh, S, L, solver, ns, n, monkeypatch):
    """The wavefront form of a smoother call (k_face_wave: un_eles claimed in reverse Cuthill-McKee
    ticket order, each sweep started once the neighbours have published their words, the iterate in
    LDS across the call) leaves the state of one launch per sweep, bit for bit -- on levels of 256,
    1,024 and 4,096 sub-elements per un_ele, with far more un_eles than co-resident workgroups
    (untitled8192 at S = 5: 8,192 level-1 un_eles over 512 workgroups), red-black and Jacobi."""
    import pamg
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))

    def run():
        g = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=solver, op=1)
        g.begin_timestep()
        g.vcycle(n)
        g.begin_timestep()
        g.vcycle(1)
        st, ov = g.state(), g.overlap()
        g.close()
        return st, ov

    monkeypatch.setenv("PAMG_FACE_PP", "0")   # the fused cycle's one-sweep calls, where the wavefront form applies
    monkeypatch.setenv("PAMG_FACE_WAVE", "0")
    monkeypatch.setenv("PAMG_FACE_CHAIN", "0")
    rs, rov = run()
    monkeypatch.setenv("PAMG_FACE_WAVE", "1")
    monkeypatch.setenv("PAMG_FACE_CHAIN", "1")
    gs, gov = run()
    assert_identical(gs, rs)
    for x, y in zip(gov, rov):
        np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,solver,ns,splits", [
    ("untitled8192.msh", 5, 3, 3, 4, ([3], [1, 2])), ("untitled8192.msh", 5, 3, 1, 4, ([2],)),
    ("untitled8192.msh", 4, 3, 3, 3, ([3], [2, 1])), ("irregular.msh", 6, 3, 3, 2, ([3], [1, 1, 1])),
    ("irregular.msh", 6, 3, 1, 5, ([2],)), ("test_sn2.msh", 4, 4, 3, 3, ([2, 1],)), ("900_ele.msh", 5, 3, 3, 4, ([2],))])
def test_face_two_sweep_passes_equal_one_sweep_launches(mesh, S, L, solver, ns, splits, monkeypatch):
    """The fused face cycle with two sweeps per HBM pass on the levels below the coarsest (k_face_pp: the
    second sweep's halo computed in the launch from the neighbours' boundary sub-elements and their down
    neighbours; level 1 one stream over the call's cycles) leaves the state of the one-sweep launches, bit
    for bit -- levels of 256, 1,024 and 4,096 sub-elements per un_ele, red-black and Jacobi, odd and even
    stream lengths, residuals at a pass's start and in its middle, calls split over time steps. Level 1's
    restrictor is folded into the pass that computes the residual it restricts (the next cycle's level-2 RHS, the
    cycle's residual itself stored only in the call's last cycle; PAMG_FACE_RR=0 keeps its own launch): both
    forms, the same state; with the fold, level 1's restrictor is launched once per call, and so is that of a coarser
    level that streams (its residual restricted into the next level's second RHS buffer, round 6)."""
    import pamg
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))

    def run(split):
        g = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=solver, op=1)
        g.timing_enable(8)   # PAMG_K_RESTRICT
        g.timing_reset()
        for n in split:
            g.begin_timestep()
            g.vcycle(n)
        st, ov = g.state(), g.overlap()
        nr = g.timing()["restrict"]["issued"]
        g.close()
        return st, ov, nr

    for split in splits:
        monkeypatch.setenv("PAMG_FACE_PP", "0")
        rs, rov, nr0 = run(split)
        monkeypatch.setenv("PAMG_FACE_PP", "3")   # both level sizes that can stream
        for rr in ("0", "1"):
            monkeypatch.setenv("PAMG_FACE_RR", rr)
            gs, gov, nr = run(split)
            assert_identical(gs, rs)
            for x, y in zip(gov, rov):
                np.testing.assert_array_equal(x, y)
            if rr == "1" and 4 ** S in (256, 1024) and L >= 2 and ns >= 2:   # level 1 streams
                # ... and so does every level 2 .. L-1 of 256 / 1,024 sub-elements whose non-final cycles are passes
                folds = 1 + (sum(4 ** (S - l + 1) in (256, 1024) for l in range(2, L)) if ns >= 3 else 0)
                assert nr == nr0 - (sum(split) - len(split)) * folds, (nr, nr0, split)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,ns,splits", [
    ("untitled8192.msh", 5, 3, 4, ([3], [1, 2])), ("untitled8192.msh", 5, 3, 2, ([2],)),
    ("900_ele.msh", 5, 3, 3, ([2, 1],)), ("irregular.msh", 5, 3, 4, ([2],))])
def test_face_chain_per_wave_equals_workgroup_chain(mesh, S, L, ns, splits, monkeypatch):
    """The coarsest level's persistent chain with its un_eles owned by waves (k_face_chain_pw: no
    workgroup barrier inside a sweep, per-wave flags) leaves the state of the workgroup chain
    (k_face_chain), bit for bit -- bench.py's op = 1 configuration (level 3: 64 sub-elements per un_ele,
    two un_eles a wave, 256 workgroups), an odd smoother length, small meshes whose last workgroup and
    waves are partly empty, calls split over time steps."""
    import pamg
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))

    def run(split):
        g = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=3, op=1)
        for n in split:
            g.begin_timestep()
            g.vcycle(n)
        st, ov = g.state(), g.overlap()
        g.close()
        return st, ov

    for split in splits:
        monkeypatch.setenv("PAMG_CHAIN_PW", "0")
        rs, rov = run(split)
        monkeypatch.setenv("PAMG_CHAIN_PW", "1")
        gs, gov = run(split)
        assert_identical(gs, rs)
        for x, y in zip(gov, rov):
            np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("mesh,S,L,solver,ns,splits", [
    ("untitled8192.msh", 5, 3, 3, 4, ([3], [1, 2])), ("untitled8192.msh", 4, 3, 1, 3, ([2],)),
    ("irregular.msh", 6, 3, 3, 3, ([2, 1],)), ("900_ele.msh", 5, 2, 3, 4, ([2],))])
def test_face_corrected_cycle_passes_equal_per_step(mesh, S, L, solver, ns, splits, monkeypatch):
    """The corrected cycle on the face operator with its smoother calls below the coarsest level as two-sweep
    passes (k_face_pp, the call's result stored as tnew -- and as tnew_nonlin in the call's last cycle -- and
    the fine residual after the cycle only in the call's last cycle) leaves the per-step sequence's state bit
    for bit (bench.py's extra.op1_cycle1 configuration first), and its level-1 calls are the passes. The residual
    and restrictor of a streaming level run as one sweep-less pass (k_face_pp res 3, the residual stored only
    where the state keeps it), and a streaming level's memset (the call from zero) and interpolation (added to
    the values the call's first pass loads) fold into its calls; PAMG_FACE_RR=0 / PAMG_FACE_FOLD=0 keep them as
    their own launches -- the same state every way."""
    import pamg
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, mesh))

    def run(split):
        g = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=solver, op=1, cycle=1)
        g.timing_enable(1 | 8)   # PAMG_K_SMOOTH_L1, PAMG_K_RESTRICT
        g.timing_reset()
        for n in split:
            g.begin_timestep()
            g.vcycle(n)
        st, ov = g.state(), g.overlap()
        tm = g.timing()
        g.close()
        return st, ov, tm["smooth_L1"]["issued"], tm["restrict"]["issued"]

    for split in splits:
        monkeypatch.setenv("PAMG_FACE_CORR_PP", "0")
        rs, rov, _, _ = run(split)
        monkeypatch.setenv("PAMG_FACE_CORR_PP", "1")
        for rr, fold in (("0", "0"), ("1", "0"), ("1", "1")):
            monkeypatch.setenv("PAMG_FACE_RR", rr)
            monkeypatch.setenv("PAMG_FACE_FOLD", fold)
            gs, gov, issued, nrestrict = run(split)
            assert_identical(gs, rs)
            for x, y in zip(gov, rov):
                np.testing.assert_array_equal(x, y)
            if 4 ** S == 1024 or 4 ** S == 256:   # level 1 streams: two calls per cycle, ceil(ns / 2) passes each
                assert issued == sum(split) * 2 * ((ns + 1) // 2), issued
                # the fused residual-restrictor: level 1's restrictor is no launch of its own
                assert nrestrict <= (L - 2 if rr == "1" else L - 1) * sum(split), (rr, nrestrict)


@pytest.mark.gpu
@pytest.mark.parametrize("cycle", [0, 1])
def test_face_chain_not_coresident_falls_back_bitwise(cycle, monkeypatch):
    """Fail-safe co-resident launches: with the handle's stream on half the GPU's CUs
    (PAMG_STREAM_CU_MASK, hipExtStreamCreateWithCUMask) the coarsest level's persistent chain -- a grid sized
    for every CU, launched after an occupancy check that cannot see the mask -- cannot be co-resident. Its
    workgroups find that out before touching anything (the arrival guard) and leave; the host then runs the
    call with one launch per sweep from the same input. bench.py's extra.op1 configuration: the state equals
    the oracle's bit for bit, and timing() reports the fallback calls."""
    monkeypatch.setenv("PAMG_STREAM_CU_MASK", "half")
    g, o = gpu_pair("untitled8192.msh", 5, 3, 3, cycle, 4)
    g.timing_reset()
    drive(g, False, cycle, steps=1, cycles=2)
    drive(o, True, cycle, steps=1, cycles=2)
    sg, so = g.state(), o.state()
    sg["t_overlap"], sg["t_overlap_old"] = g.overlap()
    so["t_overlap"], so["t_overlap_old"] = o.overlap()
    assert_identical(sg, so)
    assert g.timing()["face_fallback"]["issued"] >= 2, g.timing()["face_fallback"]
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ns,corr_pp", [(4, "0"), (2, "1")])
def test_face_chain_fallback_on_the_per_step_corrected_path(ns, corr_pp, monkeypatch):
    """the corrected cycle's per-step sequence (PAMG_FACE_CORR_PP=0, or n_smooth = 2, where the
    passes do not apply) runs the coarsest call through the gated chain too. With the stream CU-masked every such
    launch gives up and the host runs its fallback: the call must read the gates back before it returns (a
    later host wait, or a hipFree's implicit device synchronisation, would otherwise wait on a gate only the host
    opens), and a mesh re-upload right after the call must not hang. The state equals the oracle's."""
    monkeypatch.setenv("PAMG_STREAM_CU_MASK", "half")
    monkeypatch.setenv("PAMG_FACE_CORR_PP", corr_pp)
    g, o = gpu_pair("untitled8192.msh", 5, 3, 3, 1, ns)
    g.timing_reset()
    drive(g, False, 1, steps=1, cycles=2)
    drive(o, True, 1, steps=1, cycles=2)
    sg, so = g.state(), o.state()
    sg["t_overlap"], sg["t_overlap_old"] = g.overlap()
    so["t_overlap"], so["t_overlap_old"] = o.overlap()
    assert_identical(sg, so)
    assert g.timing()["face_fallback"]["issued"] >= 2, g.timing()["face_fallback"]
    # a call that leaves gates behind would deadlock here: the re-upload frees the levels (hipFree)
    g.vcycle(1)
    m = g.mesh
    g._call("pamg_upload_mesh", m.U, m.X, m.region, m.neig, m.fneig, m.dir)
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cycle", [0, 1])
def test_agglomerated_coarsest_level_follows_state_set_between_calls(cycle):
    """The agglomerated coarsest level keeps a replica of the whole level's tnew across calls;
    it is gathered from the ranks at the start of every call, so a partition's coarsest tnew written between calls
    (pamg_set_state) is what the next call starts from -- as on the single domain. Driven through pamg_run too
    (ntime 2, n_multigrid 2). 4 x-strips of untitled8192 at n_split 4, bitwise the single domain."""
    import pamg
    from pamg.solver import local_group, run_ranks
    m = pamg.Mesh.read(os.path.join(goldens.MESHES, "untitled8192.msh"))
    S, L, parts = 4, 3, 4
    owner = m.x_strip_owner(parts)
    full = pamg.SemiImplicitIterative(m, S, L, solver=3, cycle=cycle, op=1)
    ps = [pamg.SemiImplicitIterative(m, S, L, solver=3, cycle=cycle, op=1, comm=(parts, r, None, owner))
          for r in range(parts)]
    local_group(ps)
    rng = np.random.default_rng(6)
    x = rng.uniform(-1, 1, (3, full.nsub(L), m.U))

    def seq(s, own):
        s.run(2, 2)
        s.set(pamg.TNEW, L, x[:, :, own])
        s.begin_timestep()
        s.vcycle(3)
    seq(full, np.arange(m.U))
    run_ranks(ps, lambda p: seq(p, np.flatnonzero(owner == ps.index(p))))
    ref = full.state()
    for r, p in enumerate(ps):
        own = np.flatnonzero(owner == r)
        for k, v in p.state().items():
            np.testing.assert_array_equal(v, ref[k][:, :, own], err_msg=f"rank {r} {k}")
        p.close()
