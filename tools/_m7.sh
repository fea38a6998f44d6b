cd $GRAFT_REPO_ROOT
VARIANTS="E=E L1=L1 L2=L2" N=2 bash tools/ab_env.sh
