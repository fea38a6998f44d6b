cd $GRAFT_REPO_ROOT
VARIANTS="E=E G4=G4096 G3=G3072" N=2 bash tools/ab_env.sh
