# Build an A/B variant of librsgpu.so from the working tree with extra
# compiler flags (a tool, not the product):
#   bash tools/build_variant.sh NAME "-DFLAG ..."  -> tools/ab/librsgpu_NAME.so
set -e -o pipefail
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../storage-benchmarks_amd"
make -s build/enc_progs.inc build/tc_handlers.inc build/jit_prog.o build/rsgpu_capi.o build/rsgpu_host_io.o
D=/tmp/rsgpu_variant_$NAME; mkdir -p $D ../tools/ab
HF="-O3 -std=c++20 -fconstexpr-steps=50000000 -fPIC --offload-arch=gfx950 -w $FLAGS"
pids=""
for f in rs_kernels rs_bitsliced rs_tc rs_jit; do
  /opt/rocm/bin/hipcc $HF -Ibuild -c csrc/$f.hip -o $D/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc $HF -shared -o ../tools/ab/librsgpu_$NAME.so $D/rs_kernels.o $D/rs_bitsliced.o $D/rs_tc.o $D/rs_jit.o \
  build/jit_prog.o build/rsgpu_capi.o build/rsgpu_host_io.o -Wl,-soname,librsgpu.so \
  -Wl,--version-script=csrc/rsgpu.map -L/opt/rocm/lib -lhsa-runtime64
echo "built tools/ab/librsgpu_$NAME.so"
