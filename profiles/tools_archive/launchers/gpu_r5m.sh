# round 5: GPU suite after the large-M kernel (whole -m gpu suite, one process)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5m_suite.txt 2>&1; rc=$?
tail -5 gpurun_out/r5m_suite.txt
exit $rc
