set -o pipefail
bash tools/ab.sh ab9 "ns" 2 - build/libsk_npf2.so build/libsk_mu4.so build/libsk_pw3.so build/libsk_mu2.so
