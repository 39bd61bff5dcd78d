{{/*
Shared helpers of the mxtrain machine-learning charts (same file in every chart).

ml.script  -- the generated job script (SURVEY §2.3 contract): optional git clone /
              checkout / pinned commit, pre_script lines verbatim, the command and args
              of the step block each continued with " \", an echo that only runs when the
              step succeeded, post_script, clone cleanup.  No `set -e`, like the reference.
              arg: dict Values=<values> block=<"train"|"process"> done=<echo text>
ml.volumes -- config map volume (+ /dev/shm hostPath) + one PVC volume per pvc[] entry
ml.mounts  -- the matching volumeMounts
ml.resources / ml.env / ml.tolerations -- pass-throughs (env values and toleration keys
              are run through `tpl` so {{ .Release.Name }} expands)
*/}}
{{- define "ml.script" -}}
{{- $v := .Values -}}
{{- $blk := index $v .block -}}
{{- $git := $v.git | default dict -}}
#!/bin/bash
{{- if $git.repo_url }}
mkdir -p $HOME/tmp
GIT_CLONE_DIR=$HOME/tmp/$HOSTNAME
[[ -d $GIT_CLONE_DIR ]] && rm -rf $GIT_CLONE_DIR
git clone {{ $git.repo_url }} $GIT_CLONE_DIR
cd $GIT_CLONE_DIR
{{- if $git.branch }}
git checkout {{ $git.branch }}
{{- end }}
{{- if $git.commit }}
git fetch origin {{ $git.commit }}
git reset --hard {{ $git.commit }}
{{- end }}
{{- end }}
{{- range $v.pre_script }}
{{ . }}
{{- end }}
{{- range $blk.command }}
{{ . }} \
{{- end }}
{{- range $blk.args }}
{{ . }} \
{{- end }}
&& echo "{{ .done }}"
{{- range $v.post_script }}
{{ . }}
{{- end }}
{{- if $git.repo_url }}
cd $HOME
rm -rf $GIT_CLONE_DIR
{{- end }}
{{- end }}

{{- define "ml.volumes" -}}
- name: config
  configMap:
    name: {{ .cm }}
    defaultMode: 420
    items:
    - key: {{ .key }}
      path: {{ .key }}
      mode: 365
{{- if .shm }}
- name: shm
  hostPath:
    path: /dev/shm
    type: Directory
{{- end }}
{{- range $i, $pv := .pvc }}
- name: pv-{{ add $i 1 }}
  persistentVolumeClaim:
    claimName: {{ $pv.name }}
{{- end }}
{{- end }}

{{- define "ml.mounts" -}}
- name: config
  mountPath: /etc/config
{{- if .shm }}
- name: shm
  mountPath: /dev/shm
{{- end }}
{{- range $i, $pv := .pvc }}
- name: pv-{{ add $i 1 }}
  mountPath: {{ $pv.mount_path }}
{{- end }}
{{- end }}

{{- define "ml.resources" -}}
requests:
{{- range $k, $v := .requests }}
  {{ $k }}: {{ $v }}
{{- end }}
limits:
{{- range $k, $v := .limits }}
  {{ $k }}: {{ $v }}
{{- end }}
{{- end }}

{{- define "ml.env" -}}
{{- $root := .root -}}
{{- range .env }}
- name: {{ .name }}
  value: {{ tpl (toString .value) $root | quote }}
{{- end }}
{{- end }}

{{- define "ml.tolerations" -}}
{{- $root := .root -}}
{{- range .tolerations }}
- key: {{ if $.tpl_key }}{{ tpl .key $root }}{{ else }}{{ .key }}{{ end }}
{{- if .operator }}
  operator: {{ .operator | quote }}
{{- end }}
{{- if .effect }}
  effect: {{ .effect | quote }}
{{- end }}
{{- end }}
{{- end }}

{{- define "ml.annotations" -}}
karpenter.sh/do-not-disrupt: "true"
sidecar.istio.io/inject: "false"
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end }}

{{- define "ml.labels" -}}
app.kubernetes.io/name: {{ .Release.Name }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end }}
