# Round 6 v: host cost per aggregate_models call with a cached table (cfg1 MLP x 3, cfg2 ResNet-18 x 64)
set -o pipefail
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 200 python -u tools/prof_general.py 2000 mlp cached > $O/cfg1_cached.log 2>&1 || { tail -20 $O/cfg1_cached.log; exit 1; }
timeout -k 10 200 python -u tools/prof_general.py 300 resnet cached > $O/cfg2_cached.log 2>&1 || { tail -20 $O/cfg2_cached.log; exit 1; }
grep -h "us per call" $O/*.log
echo done
