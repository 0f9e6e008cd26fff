# A/B of the chunked MFMA Gram pass (k_gram_w, k > 20) at 8192^2: chunk height, columns per load,
# RinvAug in LDS vs global.  Each line: "<label> <kbench json>".
set -o pipefail
cd $GRAFT_REPO_ROOT
rm -f gpurun_out/wide_ab.txt
for k in ${KS:-33 51}; do
  for cfg in "CH=32" "CH=16 OCC=2" "CH=32 DBG=4 OCC=2" "CH=16 DBG=4 OCC=2"; do
    ch=$(echo $cfg | sed -n 's/.*CH=\([0-9]*\).*/\1/p'); bc=$(echo $cfg | sed -n 's/.*BC=\([0-9]*\).*/\1/p')
    dbg=$(echo $cfg | sed -n 's/.*DBG=\([0-9]*\).*/\1/p'); occ=$(echo $cfg | sed -n 's/.*OCC=\([0-9]*\).*/\1/p')
    echo -n "k=$k $cfg " >> gpurun_out/wide_ab.txt
    timeout -k 10 120 env GNK_GRAM_CH=$ch GNK_GRAM_BC=${bc:-0} GNK_DEBUG_GRAM=${dbg:-0} GNK_GRAM_OCC=${occ:-1} \
      python tools/kbench.py --k $k --reps 5 --kernels gram2 >> gpurun_out/wide_ab.txt || exit $?
  done
done
# correctness of the ablation variants on the k_gram_w shapes (env switches are read once per process)
for e in "GNK_GRAM_CH=16 GNK_GRAM_OCC=2" "GNK_DEBUG_GRAM=4 GNK_GRAM_OCC=2"; do
  echo "== $e" >> gpurun_out/wide_test.log
  timeout -k 10 200 env $e python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "test_gram_mfma and default and (64-47 or 64-70 or 1024-25 or 256-31 or 100-20)" >> gpurun_out/wide_test.log 2>&1 || exit $?
done
