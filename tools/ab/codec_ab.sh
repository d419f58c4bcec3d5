set -o pipefail
bash tools/gpurun_suite.sh ab 3 "base||--no-extras" "inl128k|EWDML_TOPK_INLINE=131072|--no-extras" "inl64k|EWDML_TOPK_INLINE=65536|--no-extras" "dense||--no-extras --compress none"
