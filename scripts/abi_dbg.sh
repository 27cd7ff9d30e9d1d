#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/abidbg
PAMG_DEBUG=1 timeout -k 10 60 ./examples/c_host tests/meshes/untitled8.msh 3 3 > gpurun_out/abidbg/c.txt 2>&1; echo "rc=$?" >> gpurun_out/abidbg/c.txt
PAMG_DEBUG=1 timeout -k 10 60 ./examples/c_host tests/meshes/untitled8.msh 1 1 > gpurun_out/abidbg/c1.txt 2>&1; echo "rc=$?" >> gpurun_out/abidbg/c1.txt
PAMG_DEBUG=1 timeout -k 10 60 python -c "
import sys; sys.path.insert(0,'p-a_multigrids_amd'); import pamg
s=pamg.SemiImplicitIterative(pamg.Mesh.read('tests/meshes/untitled8.msh'),1,1); s.run(1,1); print(s.get(0,1).sum()); s.close(); print('closed')
" > gpurun_out/abidbg/py.txt 2>&1; echo "rc=$?" >> gpurun_out/abidbg/py.txt
