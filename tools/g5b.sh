mkdir -p gpurun_out/g5
: > gpurun_out/g5/dbg.txt
timeout -k 10 60 ./tools/colbench 5 4 0 >> gpurun_out/g5/dbg.txt 2>&1
timeout -k 10 60 ./tools/colbench 5 0 1 >> gpurun_out/g5/dbg.txt 2>&1
cat gpurun_out/g5/dbg.txt
