set -o pipefail
bash tools/ab.sh ab10 "ns c5" 2 - build/libsk_npf2.so build/libsk_pw3.so build/libsk_np2pw3.so build/libsk_np2pw2.so
