cd /root/repo && timeout -k 10 300 python -u tools/debug_trace.py > gpurun_out/debug.log 2>&1
