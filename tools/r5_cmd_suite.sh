set -o pipefail
bash tools/r4_suite.sh r5_suite_final
