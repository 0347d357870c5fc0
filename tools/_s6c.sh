mkdir -p gpurun_out/s6c
timeout -k 10 400 python -u -m pytest tests/test_bwa_integration.py -m gpu -v --timeout 300 --timeout-method thread -k eight_contexts > gpurun_out/s6c/new.log 2>&1
echo "new rc $?"
LD_LIBRARY_PATH=$PWD/bwa-mem-harp2_amd/lib_alt timeout -k 10 400 python -u -m pytest tests/test_bwa_integration.py -m gpu -v --timeout 300 --timeout-method thread -k eight_contexts > gpurun_out/s6c/alt.log 2>&1
echo "alt rc $?"
