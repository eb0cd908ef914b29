cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
# pieces per pre-pass batch x LDS pad (caps pre-pass occupancy): cfg2 decode time
for sbp in ${SBPS:-8 16 32 64}; do for pad in ${PADS:-0 9000 22000 36000}; do
  r=$(HG_DECODE_SBP=$sbp HG_DECODE_SPEC_PAD=$pad timeout -k 10 120 python tools/decode_variants.py cfg2 2>/dev/null | grep workload) || exit 1
  echo "sbp=$sbp pad=$pad $r"
done; done
