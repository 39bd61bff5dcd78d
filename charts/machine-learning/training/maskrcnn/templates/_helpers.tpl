{{- define "mr.annotations" -}}
karpenter.sh/do-not-disrupt: "true"
sidecar.istio.io/inject: "false"
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end }}

{{- define "mr.env" -}}
- name: HOROVOD_AUTOTUNE
  value: "{{ .horovod_autotune }}"
- name: HOROVOD_LOG_LEVEL
  value: "{{ .horovod_log_level }}"
- name: NCCL_SOCKET_IFNAME
  value: "{{ .nccl_socket_ifname }}"
- name: NCCL_DEBUG
  value: "{{ .nccl_debug }}"
- name: TF_DEVICE_MIN_SYS_MEMORY_IN_MB
  value: "{{ .tf_device_min_sys_mem_mb }}"
- name: TF_CPP_MIN_LOG_LEVEL
  value: "2"
- name: TF_GPU_ALLOCATOR
  value: "cuda_malloc_async"
- name: TF_AUTOTUNE_THRESHOLD
  value: "1"
- name: TF_ENABLE_AUTO_MIXED_PRECISION
  value: "{{ .tf_enable_auto_mixed_precision }}"
- name: HSA_ENABLE_IPC_MODE_LEGACY
  value: "0"
{{- end }}

{{- define "mr.mpiargs" -}}
{{- /* MI355X: each rank pinned to disjoint cores of its GPU's NUMA node (reference: none) */}}
- -bind-to
- core
- -map-by
- slot
- -mca
- btl_tcp_if_exclude
- {{ .if_exclude }}
- -mca
- oob_tcp_if_exclude
- {{ .if_exclude }}
- -mca
- plm_rsh_no_tree_spawn
- "1"
- -x
- HOROVOD_AUTOTUNE
- -x
- HOROVOD_HIERARCHICAL_ALLREDUCE=0
- -x
- HOROVOD_HIERARCHICAL_ALLGATHER=0
- -x
- HOROVOD_TORUS_ALLREDUCE=0
- -x
- HOROVOD_LOG_LEVEL
- -x
- NCCL_SOCKET_IFNAME
- -x
- NCCL_DEBUG
- -x
- TF_DEVICE_MIN_SYS_MEMORY_IN_MB
- -x
- TF_CPP_MIN_LOG_LEVEL
- -x
- TF_GPU_ALLOCATOR
- -x
- TF_AUTOTUNE_THRESHOLD
- -x
- TF_ENABLE_AUTO_MIXED_PRECISION
- -x
- HSA_ENABLE_IPC_MODE_LEGACY
- -x
- LD_LIBRARY_PATH
- -x
- PATH
- -mca
- pml
- ob1
- -mca
- btl
- ^openib
- --display-map
- --tag-output
- --timestamp-output
{{- end }}
