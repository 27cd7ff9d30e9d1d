#!/usr/bin/env python3
"""ORACLE TEST INFRASTRUCTURE -- builds the reference Fortran as a checker.

Compiles the reference's own mode-9 path (Makefile:10 SOURCES, mode 9 =
`Semi_implicit_iterative`, transport_tri_semi.F90:14-891) with AMD flang into
`oracle/_ref/` (git-ignored; the binaries travel to the GPU box, the sources
never do). Nothing from the reference is copied into the repository: the
sources are copied into a private temporary directory, patched there, compiled,
and the temporary directory is deleted.

Patches (each is an exact, asserted string replacement):
  flang strictness (the reference was written for gfortran -freal-8-real-16):
    P1 Generic.F90 QuickSort/Partition index arrays with REAL subscripts -> int()
    P2 ShapFun.F90:39-40 REAL subscript face_nodes(...) -> int()
    P3 transport_tri.F90:374 / transport_tri_semi.F90:46 face_nodes declared
       REAL is passed to an INTEGER dummy after P2 -> declared integer
    P4 Msh2Tri.F90:167 flang's getCWD result is not blank padded -> open the
       mesh path relative to the working directory
    P5 (fp64 only) Generic.F90:23 AreEqual3 becomes ambiguous with AreEqual1
       once default real is 8 bytes -> dropped from the generic interface
  run-time configuration (values hard-coded in the reference):
    mesh path :99, n_split :118, ntime :135 and the mode-9 arguments
    (main.F90:46-47: n_multigrid, vtk_interval, solver, multi_levels, n_smooth)
    are read from `pamg_ref.nml` by oracle/ref_hooks/pamg_ref_hooks.F90
  defined start state (the reference reads memory it never initialised):
    residuale / told / RHS / source of every level (:181-186; residuale is read
    by the first restriction, :336), t_overlap_old (:198) and
    tnew_nonlin_loc2 (:545, multiplied by zero stencils at :429) := 0
  instrumentation: pamg_dump_call after each smoother / restrictor /
    get_residual / prolongator call of the first V-cycle (:331-376) and
    pamg_dump_final after the time loop (:383).

Usage: python oracle/build_ref.py [--ref /root/reference] [--out oracle/_ref]
Produces pamg_ref_fp64 (-fdefault-real-8 -fdefault-double-8: the parity
target), pamg_ref_fp32 (default real, as shipped) and
findinv_ref_fp64 (the reference's FINDInv, matrix_inversion.F90, unmodified,
behind oracle/ref_hooks/findinv_driver.F90: golden vectors of the local
block inverse, tests/make_golden_findinv.py) and csr_ref_fp64 (the reference's
csr_mul_array, matrices.F90:172-193, behind oracle/ref_hooks/csr_driver.F90:
golden vectors of the matrices.F90 SpMV, tests/make_golden_csr.py).
"""
import argparse
import os
import shutil
import subprocess
import sys
import tempfile

SOURCES = ["precision", "Structures", "Generic", "strings", "evaluate", "Msh2Tri",
           "structured_meshgen", "ShapFun", "ShapFun_unstruc", "splitting", "matrices",
           "get_vtk_files", "transport_rect", "transport_tri", "transport_tri_unstr",
           "transport_tri_semi", "amin", "main"]  # Makefile:10 order

FLANG = "/opt/rocm/lib/llvm/bin/flang"
HERE = os.path.dirname(os.path.abspath(__file__))


def sub(text, old, new, count=1, label=""):
    n = text.count(old)
    if n != count:
        raise SystemExit(f"patch {label!r}: expected {count} occurrence(s) of {old!r}, found {n}")
    return text.replace(old, new)


def sub_nth(text, old, new, nth, label=""):
    """Replace only the nth (0-based) occurrence of `old`."""
    idx = -1
    for _ in range(nth + 1):
        idx = text.find(old, idx + 1)
        if idx < 0:
            raise SystemExit(f"patch {label!r}: occurrence {nth} of {old!r} not found")
    return text[:idx] + new + text[idx + len(old):]


def patch_generic(t, fp64):
    t = sub(t, "CALL QuickSort(a(:split-1))", "CALL QuickSort(a(:int(split)-1))", label="P1a")
    t = sub(t, "CALL QuickSort(a(split:))", "CALL QuickSort(a(int(split):))", label="P1b")
    head, sep, tail = t.partition("SUBROUTINE Partition(a, marker)")
    assert sep, "P1: Partition not found"
    tail = tail.replace("a(left)", "a(int(left))").replace("a(right)", "a(int(right))")
    t = head + sep + tail
    if fp64:
        t = sub(t, "        module procedure AreEqual3\n", "", label="P5")
    return t


def patch_shapfun(t):
    t = sub(t, "tnew_loc(face_nodes(1,iface))", "tnew_loc(int(face_nodes(1,iface)))", label="P2a")
    t = sub(t, "tnew_loc(face_nodes(2,iface))", "tnew_loc(int(face_nodes(2,iface)))", label="P2b")
    return t


def patch_msh2tri(t):
    return sub(t, '      path = trim(path)//"/"//trim(filex)\n', "      path = trim(filex)\n", label="P4")


def patch_transport_tri(t):
    return sub(t, "time_det_snlx_all,face_nodes(2,3)", "time_det_snlx_all\n    integer :: face_nodes(2,3)",
               label="P3a")


def patch_semi(t):
    lines = t.splitlines(keepends=True)
    # Semi_implicit_iterative spans transport_tri_semi.F90:14-891
    assert "Subroutine Semi_implicit_iterative(" in lines[13], lines[13]
    assert "end subroutine Semi_implicit_iterative" in lines[890], lines[890]
    head, body, tail = "".join(lines[:13]), "".join(lines[13:891]), "".join(lines[891:])
    head = sub(head, "  use get_vtk_files\n", "  use get_vtk_files\n  use pamg_ref_hooks\n", label="use")
    body = sub(body, "      real :: sarea, volume, dt, L,face_nodes(2,3)\n",
               "      real :: sarea, volume, dt, L\n      integer :: face_nodes(2,3)\n", label="P3b")
    body = sub(body, "      call ReadMSH(meshList,'./Mesh_files/test_sn2.msh',ierr, totnodes)\n",
               "      call ReadMSH(meshList,trim(pamg_mesh),ierr, totnodes)\n", label="mesh")
    body = sub(body, "      n_split = 1\n", "      n_split = pamg_nsplit\n", label="n_split")
    body = sub(body, "      ntime = 2!time/dt\n", "      ntime = pamg_ntime\n", label="ntime")
    body = sub(body, "        allocate(tracer(i)%source(nloc,totele_str,totele_unst))\n",
               "        allocate(tracer(i)%source(nloc,totele_str,totele_unst))\n"
               "        tracer(i)%residuale = 0.0; tracer(i)%told = 0.0\n"
               "        tracer(i)%RHS = 0.0; tracer(i)%source = 0.0\n", label="zero-levels")
    body = sub(body, "        meshList(un_ele)%t_overlap=0.0\n",
               "        meshList(un_ele)%t_overlap=0.0\n        meshList(un_ele)%t_overlap_old=0.0\n",
               label="zero-overlap-old")
    body = sub(body, "        allocate(tnew_nonlin_loc2(nloc,4**(i_split),totele_unst,nface))\n",
               "        allocate(tnew_nonlin_loc2(nloc,4**(i_split),totele_unst,nface))\n"
               "        tnew_nonlin_loc2 = 0.0\n", label="zero-loc2")
    dump = ("            call pamg_dump_call('{tag}', ilevel, itime, multigrid, tracer, tnew_nonlin, "
            "multi_levels)\n")
    smooth = "            call smoother\n"
    assert body.count(smooth) == 3, body.count(smooth)   # :331, :352, :376
    body = sub_nth(body, smooth, smooth + dump.format(tag="smooth"), 2, label="dump-prol-smooth")
    body = sub_nth(body, smooth, smooth + dump.format(tag="smooth"), 0, label="dump-restr-smooth")
    r = "            call restrictor(tracer,totele_unst, i_split, multi_levels, ilevel)\n"
    body = sub(body, r, r + dump.format(tag="restrict"), label="dump-restrict")
    g = "            call get_residual\n"
    body = sub(body, g, g + dump.format(tag="residual"), label="dump-residual")
    c = "            ! end if\n          end do\n"
    body = sub(body, c, c + dump.format(tag="coarse").replace("            call", "          call"),
               label="dump-coarse")
    p = "            call prolongator(tracer, totele_unst, i_split, ilevel)\n"
    body = sub(body, p, p + dump.format(tag="prolong"), label="dump-prolong")
    body = sub(body, "      call CPU_TIME(t2)\n",
               "      call CPU_TIME(t2)\n      call pamg_dump_final(tracer, tnew_nonlin, meshList, "
               "multi_levels, n_split, n, k, dt, ngi, nloc, ndim)\n", label="dump-final")
    return head + body + tail


def patch_main(t):
    t = sub(t, "  use transport_tri_semi\n", "  use transport_tri_semi\n  use pamg_ref_hooks\n", label="main-use")
    t = sub(t, "  integer :: mode = 9\n", "  integer :: mode = 9\n  call pamg_cfg_read()\n", label="main-cfg")
    t = sub(t, "call Semi_implicit_iterative(1., 2, .false., 2, .025",
            "call Semi_implicit_iterative(1., 2, .false., pamg_nmultigrid, .025", label="main-nmg")
    t = sub(t, "         0., .false., 1, 5, 3, 1,4)\n",
            "         0., .false., pamg_vtk, 5, pamg_solver, pamg_levels, pamg_nsmooth)\n", label="main-args")
    return t


PATCHERS = {
    "Msh2Tri": patch_msh2tri,
    "ShapFun": patch_shapfun,
    "transport_tri": patch_transport_tri,
    "transport_tri_semi": patch_semi,
    "main": patch_main,
}


def build(ref, out, fp64, verbose=False, driver=None):
    """driver: link oracle/ref_hooks/<driver>.F90 as the program instead of the
    reference's main (csr_driver: the reference's csr_mul_array, matrices.F90:172-193)."""
    name = driver.replace("_driver", "_ref_fp64") if driver else ("pamg_ref_fp64" if fp64 else "pamg_ref_fp32")
    flags = ["-O2"] + (["-fdefault-real-8", "-fdefault-double-8"] if fp64 else [])
    tmp = tempfile.mkdtemp(prefix="pamg_refbuild_")
    try:
        for s in SOURCES:
            with open(os.path.join(ref, s + ".F90"), encoding="latin-1") as f:
                text = f.read()
            if s == "Generic":
                text = patch_generic(text, fp64)
            elif s in PATCHERS:
                text = PATCHERS[s](text)
            with open(os.path.join(tmp, s + ".F90"), "w", encoding="latin-1") as f:
                f.write(text)
        shutil.copy(os.path.join(HERE, "ref_hooks", "pamg_ref_hooks.F90"), tmp)
        order = SOURCES[:9] + ["pamg_ref_hooks"] + SOURCES[9:]
        if driver:
            shutil.copy(os.path.join(HERE, "ref_hooks", driver + ".F90"), tmp)
            order = order[:-1] + [driver]   # the driver program replaces main
        objs = []
        for s in order:
            cmd = [FLANG, "-c"] + flags + [s + ".F90", "-o", s + ".o"]
            r = subprocess.run(cmd, cwd=tmp, capture_output=True, text=True)
            if r.returncode != 0:
                sys.stderr.write(r.stdout + r.stderr)
                raise SystemExit(f"flang failed on {s}.F90")
            objs.append(s + ".o")
        os.makedirs(out, exist_ok=True)
        exe = os.path.join(os.path.abspath(out), name)
        r = subprocess.run([FLANG] + flags + objs + ["-o", exe], cwd=tmp, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise SystemExit("flang link failed")
        if verbose:
            print("built", exe)
        return exe
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def build_findinv(ref, out, verbose=False):
    """The reference's FINDInv (matrix_inversion.F90:50-148, unmodified, fp64 default real)
    behind oracle/ref_hooks/findinv_driver.F90 -> oracle/_ref/findinv_ref_fp64."""
    flags = ["-O2", "-fdefault-real-8", "-fdefault-double-8"]
    tmp = tempfile.mkdtemp(prefix="pamg_findinv_")
    try:
        shutil.copy(os.path.join(ref, "matrix_inversion.F90"), tmp)
        shutil.copy(os.path.join(HERE, "ref_hooks", "findinv_driver.F90"), tmp)
        for s in ("matrix_inversion", "findinv_driver"):
            r = subprocess.run([FLANG, "-c"] + flags + [s + ".F90", "-o", s + ".o"], cwd=tmp,
                               capture_output=True, text=True)
            if r.returncode != 0:
                sys.stderr.write(r.stdout + r.stderr)
                raise SystemExit(f"flang failed on {s}.F90")
        os.makedirs(out, exist_ok=True)
        exe = os.path.join(os.path.abspath(out), "findinv_ref_fp64")
        r = subprocess.run([FLANG] + flags + ["matrix_inversion.o", "findinv_driver.o", "-o", exe], cwd=tmp,
                           capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise SystemExit("flang link failed (findinv)")
        if verbose:
            print("built", exe)
        return exe
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "_ref"))
    ap.add_argument("--only", choices=["fp64", "fp32"], default=None)
    a = ap.parse_args()
    if not os.path.isdir(a.ref):
        raise SystemExit(f"reference not found at {a.ref}")
    for fp64 in (True, False):
        if a.only and a.only != ("fp64" if fp64 else "fp32"):
            continue
        build(a.ref, a.out, fp64, verbose=True)
    build_findinv(a.ref, a.out, verbose=True)
    build(a.ref, a.out, True, verbose=True, driver="csr_driver")


if __name__ == "__main__":
    main()
