{{/* Chart name / fullname / labels */}}
{{- define "amd-gpu-operator.name" -}}
{{- default .Chart.Name .Values.nameOverride | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "amd-gpu-operator.fullname" -}}
{{- if .Values.fullnameOverride -}}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- include "amd-gpu-operator.name" . -}}
{{- end -}}
{{- end -}}

{{- define "amd-gpu-operator.labels" -}}
app.kubernetes.io/name: {{ include "amd-gpu-operator.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" }}
{{- if .Values.operator.labels }}
{{ toYaml .Values.operator.labels }}
{{- end }}
{{- end -}}

{{/* repository/image:version, version defaulting to the chart appVersion */}}
{{- define "amd-gpu-operator.operatorImage" -}}
{{- printf "%s/%s:%s" .Values.operator.repository .Values.operator.image (.Values.operator.version | default .Chart.AppVersion) -}}
{{- end -}}

{{/* *_IMAGE fallbacks: name env value */}}
{{- define "amd-gpu-operator.imageEnv" -}}
{{- $v := index . 1 -}}
{{- if and $v.repository $v.image $v.version -}}
- name: {{ index . 0 }}
  value: {{ printf "%s/%s:%s" $v.repository $v.image $v.version | quote }}
{{- end }}
{{- end -}}
