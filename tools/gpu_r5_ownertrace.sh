set -o pipefail
O=gpurun_out/owner_trace; mkdir -p $O
for i in 1 2; do
PYTHONPATH=$PWD timeout -k 10 300 python -u tools/fwd_trace.py --so variants/trace/_C.so --params 1250000 --halos 16777216 >> $O/out.txt 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
done
MULTIGRAD_LPT=dynamic PYTHONPATH=$PWD timeout -k 10 300 python -u tools/fwd_trace.py --so variants/trace/_C.so --params 1250000 --halos 16777216 >> $O/out_dyn.txt 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
cat $O/out.txt $O/out_dyn.txt
