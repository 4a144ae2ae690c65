cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/diag_bounded.py
