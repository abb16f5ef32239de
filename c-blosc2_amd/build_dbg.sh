# Debug variants of the library (bounds-checked fast encoder, b2h_fm_debug export), selected at run
# time with B2H_LIB=c-blosc2_amd/<dir>/libblosc2.so (diagnostics only).
#   bash c-blosc2_amd/build_dbg.sh [dir (lib_dbg)] [extra flags]
set -e
H=$(cd $(dirname $0) && pwd)
D=$H/${1:-lib_dbg}
mkdir -p $D
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -fvisibility=hidden -mcode-object-version=5 -I$H/../include ${2--DB2H_FM_CHECK}"
for f in b2h_engine.hip blosc2_api.cpp b2h_frame.cpp b2h_schunk.cpp; do
  /opt/rocm/bin/hipcc $F -c -x hip $H/csrc/$f -o $D/${f%.*}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libblosc2.so $D/*.o -Wl,-soname,libblosc2.so
