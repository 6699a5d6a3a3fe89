/*
 * orc_ini.c -- TEST INFRASTRUCTURE (oracle).  ini dictionary restating the
 * semantics PINC relies on:
 *   - line grammar of iniparser 3.1 (lib/iniparser/src/iniparser.c:555-613):
 *     '#'/';' comment lines, "[section]" lower-cased, "key = value" with the
 *     value cut at the first ';' or '#' unless quoted, keys lower-cased and
 *     stored as "section:key";
 *   - PINC's list handling (src/io.c:741-841): comma separated, elements
 *     trimmed of blanks, lists repeated cyclically to the requested length;
 *   - numeric getters parse with atof so "1e6" is an integer (io.c:332-358);
 *   - setters print doubles with "%a" (io.c:447-455, 494-508) so rewriting
 *     normalised values into the dictionary is lossless;
 *   - iniApplySuffix (io.c:535-560): atof ignores the suffix, the element is
 *     multiplied by mul[i%mulLen] if it contains the suffix.
 */
#include "orc.h"
#include <ctype.h>
#include <stdarg.h>

typedef struct { char *key; char *val; } OEntry;
struct OIni { OEntry *e; int n, cap; };

void orc_die(const char *fmt, ...){
	va_list ap; va_start(ap, fmt);
	fprintf(stderr, "ORACLE ERROR: ");
	vfprintf(stderr, fmt, ap);
	fprintf(stderr, "\n");
	va_end(ap);
	exit(EXIT_FAILURE);
}

static char *dupstr(const char *s){
	size_t n = strlen(s);
	char *r = malloc(n + 1);
	memcpy(r, s, n + 1);
	return r;
}

static void lower(char *s){ for(; *s; s++) *s = (char)tolower((unsigned char)*s); }

/* strip leading/trailing whitespace in place, return start */
static char *strip(char *s){
	while(*s && isspace((unsigned char)*s)) s++;
	char *e = s + strlen(s);
	while(e > s && isspace((unsigned char)e[-1])) e--;
	*e = '\0';
	return s;
}

void oini_set(OIni *ini, const char *key, const char *value){
	char *k = dupstr(key);
	lower(k);
	for(int i = 0; i < ini->n; i++){
		if(!strcmp(ini->e[i].key, k)){
			free(ini->e[i].val);
			ini->e[i].val = dupstr(value);
			free(k);
			return;
		}
	}
	if(ini->n == ini->cap){
		ini->cap = ini->cap ? 2*ini->cap : 64;
		ini->e = realloc(ini->e, ini->cap*sizeof(*ini->e));
	}
	ini->e[ini->n].key = k;
	ini->e[ini->n].val = dupstr(value);
	ini->n++;
}

static void parse_line(OIni *ini, char *raw, char *section){
	char *line = strip(raw);
	size_t len = strlen(line);
	if(len == 0 || line[0] == '#' || line[0] == ';') return;
	if(line[0] == '[' && line[len-1] == ']'){
		line[len-1] = '\0';
		char *sec = strip(line + 1);
		strcpy(section, sec);
		lower(section);
		return;
	}
	char *eq = strchr(line, '=');
	if(!eq) return; /* syntax error lines are ignored by the reference loader */
	*eq = '\0';
	char *key = strip(line);
	char *val = strip(eq + 1);
	if(val[0] == '"' || val[0] == '\''){
		char q = val[0];
		char *end = strchr(val + 1, q);
		if(end){ *end = '\0'; val = val + 1; }
	} else {
		char *c = strpbrk(val, ";#");
		if(c) *c = '\0';
		val = strip(val);
	}
	char full[512];
	snprintf(full, sizeof(full), "%s:%s", section, key);
	oini_set(ini, full, val);
}

OIni *oini_from_string(const char *text){
	OIni *ini = calloc(1, sizeof(*ini));
	char section[256] = "";
	char *copy = dupstr(text);
	char *save = NULL;
	for(char *ln = strtok_r(copy, "\n", &save); ln; ln = strtok_r(NULL, "\n", &save))
		parse_line(ini, ln, section);
	free(copy);
	return ini;
}

OIni *oini_load(const char *path){
	FILE *f = fopen(path, "rb");
	if(!f) orc_die("cannot open %s", path);
	fseek(f, 0, SEEK_END);
	long n = ftell(f);
	fseek(f, 0, SEEK_SET);
	char *buf = malloc(n + 1);
	if(fread(buf, 1, n, f) != (size_t)n) orc_die("short read %s", path);
	buf[n] = '\0';
	fclose(f);
	OIni *ini = oini_from_string(buf);
	free(buf);
	return ini;
}

void oini_free(OIni *ini){
	if(!ini) return;
	for(int i = 0; i < ini->n; i++){ free(ini->e[i].key); free(ini->e[i].val); }
	free(ini->e);
	free(ini);
}

static const char *lookup(const OIni *ini, const char *key){
	char k[512];
	snprintf(k, sizeof(k), "%s", key);
	lower(k);
	for(int i = 0; i < ini->n; i++) if(!strcmp(ini->e[i].key, k)) return ini->e[i].val;
	return NULL;
}

int oini_has(const OIni *ini, const char *key){ return lookup(ini, key) != NULL; }

const char *oini_raw(const OIni *ini, const char *key){
	const char *v = lookup(ini, key);
	if(!v) orc_die("Key \"%s\" not found in input file", key);
	return v;
}

int oini_nelem(const OIni *ini, const char *key){
	const char *v = oini_raw(ini, key);
	if(v[0] == '\0') return 0;
	int n = 1;
	for(; *v; v++) n += (*v == ',');
	return n;
}

int oini_int(const OIni *ini, const char *key){ return (int)atof(oini_raw(ini, key)); }
long oini_long(const OIni *ini, const char *key){ return (long)atof(oini_raw(ini, key)); }
double oini_double(const OIni *ini, const char *key){ return atof(oini_raw(ini, key)); }

/* split on ',' and trim blanks (only ' ', as io.c:785-786) */
static char **split(const char *list, int *count){
	int cap = 2;
	for(const char *t = list; *t; t++) cap += (*t == ',');
	char **res = malloc(cap*sizeof(char*));
	int n = 0;
	const char *start = list;
	for(const char *t = list;; t++){
		if(*t == ',' || *t == '\0'){
			const char *a = start, *b = t - 1;
			while(*a == ' ' && a < b) a++;
			while(*b == ' ' && a < b) b--;
			int len = (int)(b - a + 1);
			if(len < 0) len = 0;
			res[n] = malloc(len + 1);
			memcpy(res[n], a, len);
			res[n][len] = '\0';
			n++;
			start = t + 1;
			if(*t == '\0') break;
		}
	}
	res[n] = NULL;
	*count = n;
	return res;
}

void oini_freestrarr(char **arr){
	for(int i = 0; arr[i]; i++) free(arr[i]);
	free(arr);
}

char **oini_strarr(const OIni *ini, const char *key, int n){
	int m;
	char **base = split(oini_raw(ini, key), &m);
	char **res = malloc((n + 1)*sizeof(char*));
	for(int i = 0; i < n; i++) res[i] = dupstr(base[i % m]);
	res[n] = NULL;
	oini_freestrarr(base);
	return res;
}

int *oini_intarr(const OIni *ini, const char *key, int n){
	char **s = oini_strarr(ini, key, n);
	int *r = malloc(n*sizeof(int));
	for(int i = 0; i < n; i++) r[i] = (int)atof(s[i]);
	oini_freestrarr(s);
	return r;
}

long *oini_longarr(const OIni *ini, const char *key, int n){
	char **s = oini_strarr(ini, key, n);
	long *r = malloc(n*sizeof(long));
	for(int i = 0; i < n; i++) r[i] = (long)atof(s[i]);
	oini_freestrarr(s);
	return r;
}

double *oini_doublearr(const OIni *ini, const char *key, int n){
	char **s = oini_strarr(ini, key, n);
	double *r = malloc(n*sizeof(double));
	for(int i = 0; i < n; i++) r[i] = atof(s[i]);
	oini_freestrarr(s);
	return r;
}

void oini_setdoublearr(OIni *ini, const char *key, const double *v, int n){
	char list[2048] = "";
	char num[64];
	for(int i = 0; i < n; i++){
		snprintf(num, sizeof(num), i ? ",%a" : "%a", v[i]);
		strcat(list, num);
	}
	oini_set(ini, key, list);
}

void oini_setdouble(OIni *ini, const char *key, double v){
	char num[64];
	snprintf(num, sizeof(num), "%a", v);
	oini_set(ini, key, num);
}

void oini_scaledouble(OIni *ini, const char *key, double factor){
	int n = oini_nelem(ini, key);
	double *a = oini_doublearr(ini, key, n);
	for(int i = 0; i < n; i++) a[i] *= factor;
	oini_setdoublearr(ini, key, a, n);
	free(a);
}

void oini_applysuffix(OIni *ini, const char *key, const char *suffix,
                      const double *mul, int mullen){
	int n = oini_nelem(ini, key);
	char **s = oini_strarr(ini, key, n);
	double *a = malloc(n*sizeof(double));
	for(int i = 0; i < n; i++){
		a[i] = atof(s[i]);
		if(strstr(s[i], suffix)) a[i] *= mul[i % mullen];
	}
	oini_setdoublearr(ini, key, a, n);
	free(a);
	oini_freestrarr(s);
}
