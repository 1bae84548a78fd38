# round-3 session: parity of the scan/base change and the tx fast path,
# scan chunks-per-thread A/B, c3 LDS-DMA A/B, tx timing on rotating buffers
TESTS="tests/test_gpu_scatter.py tests/test_gpu_volume.py tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_group.py" bash tools/gpu.sh r03i tests || exit 1
for k in 4 2 1; do
  USN_SCAN_CPT=$k SCB_CFGS="c5 c2" bash tools/gpu.sh r03i scb || exit 1
  mv gpurun_out/r03i/scb_c5.log gpurun_out/r03i/scb_c5_cpt$k.log
  mv gpurun_out/r03i/scb_c2.log gpurun_out/r03i/scb_c2_cpt$k.log
done
TXB_ARGS="1048576 40 1 --rotate 6" bash tools/gpu.sh r03i txbench || exit 1
ABL_CFGS=c3 ABL_VARIANTS="base c3glds" bash tools/gpu.sh r03i abl
