# Build libkdstep.so variants that differ only in k_loss_grad's geometry (-D KD_LG_NT/U/ROWS),
# for tools/gpu_loss_cfg.sh.  Usage: bash tools/build_loss_variants.sh "NT:U:ROWS ..."
set -e
cd "$(dirname "$0")/.."
CS=knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd/csrc
for cfg in $1; do
  IFS=: read nt u rows <<< "$cfg"
  d=tools/variants/lg_${nt}_${u}_${rows}; mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -Iinclude \
      -DKD_LG_NT=$nt -DKD_LG_U=$u -DKD_LG_ROWS=$rows -c $CS/kd_loss.hip -o $d/kd_loss.o
  objs=$(ls $CS/build/*.o | grep -v kd_loss.o)
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $objs $d/kd_loss.o -o $d/libkdstep.so
  rm $d/kd_loss.o
  echo built $d
done
