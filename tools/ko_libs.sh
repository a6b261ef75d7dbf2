# Knock-out library variants (timing only, wrong results) for tools/ko_bench.sh
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
for v in ${VARIANTS:-base: fft:-DTFHE_KO_FFT bar:-DTFHE_KO_BAR mac:-DTFHE_KO_MAC inv:-DTFHE_KO_INV tmp:-DTFHE_KO_TMP dig:-DTFHE_KO_DIG}; do
  name=${v%%:*}; flags=${v#*:}
  rm -rf /tmp/ko_$name && mkdir -p /tmp/ko_$name
  make -s -C zig-tfhe_amd OUT=/tmp/ko_$name EXTRA="$flags" -j8 >/dev/null
  cp /tmp/ko_$name/libtfhe_gpu.so tools/bin/libko_$name.so
done
