set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/grad_diag2.log
: > $O
timeout -k 10 200 python tools/grad_diag.py fp32 fp32-nocudnn torch-bf16 fused-bf16 >> $O 2>&1 || exit $?
DIAG_TAG=nowino MIOPEN_DEBUG_CONV_WINOGRAD=0 timeout -k 10 200 python tools/grad_diag.py fp32 >> $O 2>&1 || exit $?
DIAG_TAG=nofft_nowino MIOPEN_DEBUG_CONV_WINOGRAD=0 MIOPEN_DEBUG_CONV_FFT=0 timeout -k 10 200 python tools/grad_diag.py fp32 >> $O 2>&1 || exit $?
DIAG_TAG=gemmonly MIOPEN_DEBUG_CONV_WINOGRAD=0 MIOPEN_DEBUG_CONV_FFT=0 MIOPEN_DEBUG_CONV_DIRECT=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 timeout -k 10 200 python tools/grad_diag.py fp32 >> $O 2>&1 || exit $?
