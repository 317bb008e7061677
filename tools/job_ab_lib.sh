set -o pipefail
bash tools/ab_env.sh gpurun_out/ablib 2 "-" "VIT_FWD_LIB=1" "VIT_FWD_LIB=2" "VIT_DGRAD_LIB=1" "VIT_FWD_LIB=1 VIT_DGRAD_LIB=1"
for f in gpurun_out/ablib/ab_*_1.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['config']['final_loss'])" $f; done
