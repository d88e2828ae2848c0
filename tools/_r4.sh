set -o pipefail
bash tools/_r3.sh || exit 1
bash tools/_nt.sh nt1 ns - build/libsk_ntst.so build/libsk_ntall.so || exit 1
bash tools/ab.sh ab4 "ns" 1 build/libsk_ntst.so build/libsk_ntall.so
