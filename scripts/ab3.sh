set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for f in scripts/ablibs/lib_cur.so scripts/ablibs/lib_conc.so; do
  PAMG_LIB=$PWD/$f timeout -k 10 60 python scripts/vc_wall.py 5 > gpurun_out/ab.txt 2>&1 || exit 1
  echo "$(basename $f):"; grep -v amdgpu gpurun_out/ab.txt
done
