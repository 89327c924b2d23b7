# round 6: attention keys per split 256 / 512 (one split per item at the text steps' ~200-key contexts) vs the default
cd $GRAFT_REPO_ROOT
SWEEP='FO_ATTN_KPS=0|FO_ATTN_KPS=256|FO_ATTN_KPS=512' bash scripts/gpu_call.sh r06zg sweep
