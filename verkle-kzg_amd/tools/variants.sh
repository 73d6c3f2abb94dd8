set -e
cd $GRAFT_REPO_ROOT/verkle-kzg_amd
for l in 1 2 4 8; do
  echo "== LSEG=$l"
  VKZG_MSM_LSEG=$l timeout -k 10 100 python3 tools/msm_probe.py | head -1
  VKZG_MSM_LSEG=$l timeout -k 10 100 python3 tools/scale_probe.py | grep "part=0" | cut -c1-30
done
