cd $GRAFT_REPO_ROOT && export PYTHONPATH=$GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 400 python bench/probe_search.py > gpurun_out/probe1.log 2>&1
