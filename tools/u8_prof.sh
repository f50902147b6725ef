set -e
O=gpurun_out/r03_u8
mkdir -p $O
timeout -k 10 60 ab/knn_lab_base 4096 61 625 4506 20 > $O/lab.txt 2>&1
R=$PWD; cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- ab/knn_lab_base 4096 61 625 4506 5 > $O/prof.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc1 -o run -- ab/knn_lab_base 4096 61 625 4506 2 > $O/pmc1.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc2 -o run -- ab/knn_lab_base 4096 61 625 4506 2 > $O/pmc2.txt 2>&1
echo done
