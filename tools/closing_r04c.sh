set -o pipefail
bash tools/closing.sh 1 && TAG=r04fin3 tools/gpu.sh profdriver
