# Round 6 check 4: onesweep block shapes around 512 x 12 (exp/D) — E 512 x 16, F (1024 x 16 histogram), G 512 x 8.
set -u
export TMPDIR=/tmp
VARIANTS="D E F G" N=2 bash tools/ab.sh || exit 1
