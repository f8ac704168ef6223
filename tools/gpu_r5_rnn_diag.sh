#!/bin/bash
# Round 5: what each part of the recurrence step costs (libftmi_diag.so timing switches,
# tools/rnn_diag.py; results invalid under bits 2/32/64/128, timing only; -1 = a timeout).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export FTMI_LIB=forwardtacotron_amd/libftmi_diag.so
export DIAG_ENVS="FTMI_RNN_DIAG=0;FTMI_RNN_U8=0;FTMI_RNN_DIAG=2;FTMI_RNN_DIAG=34;FTMI_RNN_DIAG=66;FTMI_RNN_DIAG=130;FTMI_RNN_DIAG=226;FTMI_RNN_DIAG=0;FTMI_RNN_U8=0"
timeout -k 10 500 python -u tools/rnn_diag.py > gpurun_out/${OUT:-r5}_rnn_diag.txt 2>&1
rc=$?; cat gpurun_out/${OUT:-r5}_rnn_diag.txt; exit $rc
