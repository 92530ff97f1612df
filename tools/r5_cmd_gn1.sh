set -o pipefail
T=gpurun_out/r5_gn1; mkdir -p $T
timeout -k 10 60 python -u tools/diag_empty_capture.py > $T/diag_empty_capture.log 2>&1; echo "[empty capture] rc=$?"
timeout -k 10 400 python -u -m pytest tests/test_netops.py tests/test_abi.py -m gpu -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1; rc=$?
tail -2 $T/tests.log; grep -E "^(FAILED|ERROR)" $T/tests.log | head
trc=$rc
PROF=1 bash tools/r5_ab.sh r5_gn1 kitti-packnet-san 2 "rpt8:" "rpt4:PSFM_GN_RES_RPT=4@@" || exit $?
bash tools/r5_ab.sh r5_gn1 kitti-packnet 1 "rpt8:" "rpt4:PSFM_GN_RES_RPT=4@@"
exit ${trc:-0}
