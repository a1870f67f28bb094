set -o pipefail
LIBS="base xko1 xko2 xko3 g9o1" ROUNDS=2 PREFILL=1 bash tools/r5_ab.sh
