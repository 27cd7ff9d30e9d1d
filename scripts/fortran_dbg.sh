#!/bin/bash
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/fdbg && cd $R/gpurun_out/fdbg
cp $R/tests/meshes/untitled8.msh .
for cs in 1 0; do for dump in "'out.bin'" "''"; do
printf "&transport mesh_file='untitled8.msh', n_split=1, multi_levels=1, n_smooth=4, solver=3, ntime=1, n_multigrid=1, device=0, dump=$dump, call_sites=$cs /\n" > pamg_run.nml
PAMG_DEBUG=1 timeout -k 10 60 $R/p-a_multigrids_amd/bin/pamg_transport > log_${cs}_${#dump}.txt 2>&1
echo "rc=$?" >> log_${cs}_${#dump}.txt
done; done
cd $R && PAMG_C_OVERLAP=1 PAMG_DEBUG=1 timeout -k 10 60 ./examples/c_host tests/meshes/untitled8.msh 1 1 > gpurun_out/fdbg/c_ov.txt 2>&1; echo "rc=$?" >> gpurun_out/fdbg/c_ov.txt
