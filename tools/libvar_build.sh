# Library variants for A/B and knock-out timing: each NAME:FLAGS builds the whole
# library with EXTRA=FLAGS in its own directory and copies it to tools/bin/lib_NAME.so.
#   VARIANTS="base: ex2r:-DTFHE_DUO_EX2_REGS=1" bash tools/libvar_build.sh
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//,/ }
  ( make -s -C zig-tfhe_amd OUT=/tmp/libvar_$name EXTRA="$flags" /tmp/libvar_$name/libtfhe_gpu.so >/dev/null 2>&1 \
      && cp /tmp/libvar_$name/libtfhe_gpu.so tools/bin/lib_$name.so && echo "built $name" ) &
done
wait
