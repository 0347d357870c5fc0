# round-6 scratch driver: headline step A/B/A -- HEAD library vs the c9459fb build (lib_alt)
mkdir -p gpurun_out/s6u
Q="bench:--side-stages,0,--cpu-seconds,0,--e2e-reads,0,--other-profile,0,--parity,0"
bash tools/gpu_run.sh s6u "$Q" || exit 1
SMEMGPU_LIB=$PWD/bwa-mem-harp2_amd/lib_alt/libsmemgpu.so bash tools/gpu_run.sh s6u_alt "$Q" || exit 1
bash tools/gpu_run.sh s6u2 "$Q" && echo "ALL OK s6u"
