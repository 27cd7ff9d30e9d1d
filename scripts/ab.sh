# A/B timing of library builds under scripts/ablibs (PAMG_LIB override), same box
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for rep in 1 2; do
for f in scripts/ablibs/*.so; do
  PAMG_LIB=$PWD/$f timeout -k 10 60 python scripts/vc_probe.py ${VC_CASES:-5,3,4,15} > gpurun_out/ab.txt 2>&1 || exit 1
  echo "$(basename $f): $(grep -v amdgpu gpurun_out/ab.txt)"
done
done
