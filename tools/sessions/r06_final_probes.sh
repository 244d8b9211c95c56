set -u
mkdir -p gpurun_out/r06/final_probes
timeout -k 10 120 python -u tools/first_chunk_probe.py --admissions 50 > gpurun_out/r06/final_probes/fcp_2_8.json 2>&1 || { echo fcp failed; tail -5 gpurun_out/r06/final_probes/fcp_2_8.json; exit 1; }
tail -1 gpurun_out/r06/final_probes/fcp_2_8.json
for i in 1 2 3; do timeout -k 10 120 python -u tools/race_probe.py --jobs 80 >> gpurun_out/r06/final_probes/race_product.txt 2>&1 || { echo race failed; exit 1; }; done
cat gpurun_out/r06/final_probes/race_product.txt
