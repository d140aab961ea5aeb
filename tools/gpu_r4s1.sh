bash tools/gpu_session.sh r4s1 || exit $?
cd tools
L=../hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so
timeout -k 10 200 python ab_attn_libs.py $L $L $L $L --qs 0,1,2,3 --vt 1,3 --reps 6 > ../gpurun_out/r4s1/ab_fwd_vt.log 2>&1 || exit $?
tail -4 ../gpurun_out/r4s1/ab_fwd_vt.log
timeout -k 10 300 python ab_attn_libs.py ../ab/lib_abase.so ../ab/lib_aq3.so ../ab/lib_as3.so ../ab/lib_axq.so ../ab/lib_axq3.so ../ab/lib_abase.so ../ab/lib_aq3.so ../ab/lib_as3.so ../ab/lib_axq.so ../ab/lib_axq3.so --bwd --qs 0,1,2,3,4,5,6,7,8,9 --reps 3 > ../gpurun_out/r4s1/ab_bwd.log 2>&1 || exit $?
tail -4 ../gpurun_out/r4s1/ab_bwd.log
