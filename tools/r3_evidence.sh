# Round-3 evidence at one commit (GPU box): part A (decode PMC per shape),
# then part B (compaction PMC, headline profile, smoke + GPU tests + bench).
cd "$GRAFT_REPO_ROOT" && bash tools/r3_evidence_a.sh && bash tools/r3_evidence_b.sh
