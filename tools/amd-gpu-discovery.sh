#!/usr/bin/env bash
# amd-gpu-discovery.sh -- GPU discovery for Flink's external-resource framework on MI355X nodes.
#
# Drop-in for the discovery script Flink's GPUDriver runs
# (flink-external-resources/flink-external-resource-gpu/.../GPUDriver.java:72-91, which executes the
# configured script with "<amount> <args>" and reads comma-separated device indices from stdout;
# reference script: nvidia-gpu-discovery.sh + gpu-discovery-common.sh).  Same command line:
#
#   amd-gpu-discovery.sh <gpu-amount> [--enable-coordination-mode] [--coordination-file <path>]
#
# Prints the HIP device ordinals the TaskManager may use ("0,1,..."); each GpuWindowOperator subtask
# passes one of them as gwo_config.device (hipSetDevice).  Devices come from the KFD topology in sysfs
# (nodes with SIMDs are GPUs, in HIP ordinal order), so no SMI tool is needed; HIP_VISIBLE_DEVICES, when
# set, restricts and renumbers them the way the HIP runtime does.  In coordination mode a lock-protected
# file records "<index> <pid>" per occupied device, so TaskManagers on one host never share a GPU; an
# entry whose process has exited is reclaimed.  Exit status 1 when not enough devices are free.
set -u

TOPOLOGY=${GWO_KFD_TOPOLOGY:-/sys/class/kfd/kfd/topology/nodes}

usage() {
  echo "Usage: $0 gpu-amount [--enable-coordination-mode] [--coordination-file filePath]" >&2
  exit 1
}

[ $# -ge 1 ] || usage
amount=$1
shift
case $amount in '' | *[!0-9]*) usage ;; esac
coordinate=0
coord_file=/var/tmp/flink-gpu-coordination
while [ $# -gt 0 ]; do
  case $1 in
    --enable-coordination-mode) coordinate=1 ;;
    --coordination-file) shift; [ $# -gt 0 ] || usage; coord_file=$1 ;;
    *) ;;   # unknown options are ignored, as the reference script does
  esac
  shift
done
[ "$amount" -eq 0 ] && exit 0

# HIP ordinals: KFD nodes with SIMDs (CPU nodes report simd_count 0), by node number.
list_devices() {
  local n=0 node
  for node in $(ls -d "$TOPOLOGY"/[0-9]* 2>/dev/null | sort -t/ -k1 -V); do
    local simds
    simds=$(awk '$1 == "simd_count" {print $2}' "$node/properties" 2>/dev/null)
    if [ -n "$simds" ] && [ "$simds" -gt 0 ]; then
      echo $n
      n=$((n + 1))
    fi
  done
}

mapfile -t all < <(list_devices)
if [ -n "${HIP_VISIBLE_DEVICES:-}" ]; then
  # visible devices are renumbered 0..k-1 in the listed order
  IFS=',' read -r -a vis <<< "$HIP_VISIBLE_DEVICES"
  all=()
  for i in "${!vis[@]}"; do all+=("$i"); done
fi
if [ ${#all[@]} -eq 0 ]; then
  echo "No AMD GPU found in $TOPOLOGY." >&2
  exit 1
fi

emit() { local IFS=','; echo "$*"; }

if [ $coordinate -eq 0 ]; then
  if [ "$amount" -gt ${#all[@]} ]; then
    echo "Could not get enough GPU resources." >&2
    exit 1
  fi
  emit "${all[@]:0:$amount}"
  exit 0
fi

owner=$PPID   # the TaskManager that runs this script holds the devices
touch "$coord_file" 2>/dev/null || { echo "Cannot write $coord_file." >&2; exit 1; }
exec 9<>"$coord_file.lock"
flock -x 9
declare -A held=()
while read -r idx pid; do
  [ -n "${idx:-}" ] || continue
  if [ -n "${pid:-}" ] && kill -0 "$pid" 2>/dev/null; then held[$idx]=$pid; fi   # drop dead owners
done < "$coord_file"
picked=()
for i in "${all[@]}"; do
  [ ${#picked[@]} -ge "$amount" ] && break
  [ -n "${held[$i]:-}" ] || picked+=("$i")
done
if [ ${#picked[@]} -lt "$amount" ]; then
  echo "Could not get enough GPU resources." >&2
  exit 1
fi
{
  for i in "${!held[@]}"; do echo "$i ${held[$i]}"; done
  for i in "${picked[@]}"; do echo "$i $owner"; done
} > "$coord_file.tmp" && mv "$coord_file.tmp" "$coord_file"
emit "${picked[@]}"
