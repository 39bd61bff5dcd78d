{{- define "ml.annotations" -}}
karpenter.sh/do-not-disrupt: "true"
sidecar.istio.io/inject: "false"
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end }}
