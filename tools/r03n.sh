# round-3 session: kernel breakdown of the bench (all configs) and of the tx
# rings; A/B of the scatter's grouped write-out
SCB_CFGS="c5 c2" SCB_VARIANTS="base scg0" bash tools/gpu.sh r03n scb || exit 1
bash tools/gpu.sh r03n rocprof || exit 1
TXB_ARGS="1048576 24 1 --rotate 6" bash tools/gpu.sh r03n txprof
