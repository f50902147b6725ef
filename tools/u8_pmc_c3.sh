set -u
O=gpurun_out/r05_aw; mkdir -p $O
timeout -k 10 60 ab/knn_lab_base 500 61 2500 550 20 > $O/lab.txt 2>&1 || exit 1
R=$PWD; cd /tmp && export TMPDIR=/tmp && cd $R
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc1 -o run -- ab/knn_lab_base 500 61 2500 550 2 > $O/pmc1.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc2 -o run -- ab/knn_lab_base 500 61 2500 550 2 > $O/pmc2.txt 2>&1 || exit 1
echo done
