set -o pipefail
bash tools/closing.sh 1 && bash tools/closing.sh 2
