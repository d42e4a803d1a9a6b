set -u
mkdir -p gpurun_out/drv
for i in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/drv/a$i.json > /dev/null 2>&1 || exit 1; python -c "import json;d=json.load(open('gpurun_out/drv/a$i.json'));print('w5 s20', d['ms_per_step'])"; done
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 50 --no-wisdm --out gpurun_out/drv/b$i.json > /dev/null 2>&1 || exit 1; python -c "import json;d=json.load(open('gpurun_out/drv/b$i.json'));print('w50 s20 nowisdm', d['ms_per_step'])"; done
for i in 1 2; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --graph 1 --no-wisdm --out gpurun_out/drv/c$i.json > /dev/null 2>&1 || exit 1; python -c "import json;d=json.load(open('gpurun_out/drv/c$i.json'));print('graph w5 s20', d['ms_per_step'])"; done
for i in 1; do timeout -k 10 200 python bench.py --gpus 1 --steps 500 --warmup 20 --no-wisdm --out gpurun_out/drv/d$i.json > /dev/null 2>&1 || exit 1; python -c "import json;d=json.load(open('gpurun_out/drv/d$i.json'));print('w20 s500', d['ms_per_step'])"; done
