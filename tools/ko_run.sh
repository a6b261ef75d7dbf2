set -o pipefail
for f in tools/bin/ko_*; do
  echo "== $f"; timeout -k 10 60 $f 1024 | grep "rep 1" || exit 1
  echo "== $f split"; TFHE_BR_KERNEL=split timeout -k 10 60 $f 1024 | grep "rep 1" || exit 1
done
