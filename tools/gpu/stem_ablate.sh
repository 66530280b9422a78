# stem forward ablation libraries (python csrc/build.py --define STEM_ABLATE=N for N in 1 2 4 3 first)
# vs the release library: bash tools/gpu/stem_ablate.sh -> gpurun_out/stemab/r.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stemab
N=mil_nce_howto100m_amd/_native
timeout -k 10 120 python tools/stem_fwd_ab.py > gpurun_out/stemab/r.log 2>&1 || exit 1
for d in 1 2 4 3; do
  MILNCE_LIB_PATH=$N/libmilnce_hip_def_STEM_ABLATE=$d.so timeout -k 10 120 python tools/stem_fwd_ab.py >> gpurun_out/stemab/r.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/stem_fwd_ab.py >> gpurun_out/stemab/r.log 2>&1
