# floor microkernel (exact + fast modes) and the timing-events A/B with the stride
bash tools/run/floor.sh || exit $?
bash tools/run/events_ab.sh
