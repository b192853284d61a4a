cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in old new old new; do
  timeout -k 5 60 build/kbench_$v 32768 8 960 >> gpurun_out/kb.txt 2>&1 || exit 3
  timeout -k 5 60 build/kbench_$v 8192 16 1920 0 0 8 0 2 >> gpurun_out/kb.txt 2>&1 || exit 3
done
cat gpurun_out/kb.txt
