set -u
bash tools/diag_run.sh k_describe default seg2 seg4 seg6 default seg4
