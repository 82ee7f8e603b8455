# single-proof latency through the host boundary: Python with torch's HIP runtime, Python with
# /opt/rocm's (what the JS addon loads), and the JS module itself (every sample)
set -e
timeout -k 10 120 python -u profiles/hip_runtime_ab.py torch 20 7
timeout -k 10 120 python -u profiles/hip_runtime_ab.py notorch 20 7
timeout -k 10 120 python -u profiles/hip_runtime_ab.py torch 20 7
timeout -k 10 120 python -u profiles/hip_runtime_ab.py notorch 20 7
KGS_JS_TIME_ALL=1 KGS_JS_CONTEXTS=8 timeout -k 10 200 node --expose-gc kzg-grandsums-study_amd/js/test/time_prove.js /tmp/kgs_bench_p20.ptau 20 7
