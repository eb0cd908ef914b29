# Round 4: compaction record gather with adjacent pieces per lane (adj2, adj4).
set -e
timeout -k 10 500 bash tools/ab_compact.sh base adj2 adj4 | grep "^==\|encode_records"
