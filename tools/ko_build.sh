# Development: knock-out variants of the blind-rotation kernel for timing (tools/phase_prof.hip)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
VARIANTS=${VARIANTS:-"base: fft:-DTFHE_KO_FFT bar:-DTFHE_KO_BAR mac:-DTFHE_KO_MAC inv:-DTFHE_KO_INV tmp:-DTFHE_KO_TMP"}
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DTFHE_PHASE_PROF ${flags} \
      -Izig-tfhe_amd/csrc -o tools/bin/ko_$name tools/phase_prof.hip 2>/dev/null &
done
wait
