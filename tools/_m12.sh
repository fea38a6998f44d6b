cd $GRAFT_REPO_ROOT
VARIANTS="E=E W3=W3 W4=W4" N=2 bash tools/ab_env.sh
