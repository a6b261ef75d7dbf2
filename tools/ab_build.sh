# Build tools/bin/libA.so from the committed tree and tools/bin/libB.so from the working tree.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
make -C zig-tfhe_amd -j8 >/dev/null && cp zig-tfhe_amd/lib/libtfhe_gpu.so tools/bin/libB.so
git stash -q
make -C zig-tfhe_amd -j8 >/dev/null && cp zig-tfhe_amd/lib/libtfhe_gpu.so tools/bin/libA.so
git stash pop -q
make -C zig-tfhe_amd -j8 >/dev/null
