bash tools/gpu_iter.sh 200 256 && bash tools/gpu_var.sh 200 256 build/libsk_pw1.so build/libsk_pw3.so build/libsk_pw2mu2.so build/libsk_pw2mu4.so
