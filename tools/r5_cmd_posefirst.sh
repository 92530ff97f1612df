set -o pipefail
PROF=1 bash tools/r5_ab.sh r5_posefirst kitti-resnet-san 3 "posefirst:--pose-first" "poseafter:"
