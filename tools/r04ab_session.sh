# k_encode switch A/B (ABBA): memo window 4, probe groups 2 / 4, on C1 and C5
set -o pipefail
bash tools/ab.sh 1 5
