set -o pipefail
bash tools/r5_final.sh r5_finalB kitti-packnet ddad-packnet-san
