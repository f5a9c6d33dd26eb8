/* conf.c -- see conf.h */
#include "conf.h"

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static char *trim(char *s) {
    while (*s && isspace((unsigned char)*s)) ++s;
    char *e = s + strlen(s);
    while (e > s && isspace((unsigned char)e[-1])) *--e = '\0';
    return s;
}

int dsort_conf_read(const char *path, int need_ip, dsort_conf *out) {
    memset(out, 0, sizeof(*out));
    FILE *f = fopen(path, "r");
    if (!f) {
        fprintf(stderr, "conf: cannot open %s\n", path);
        return -1;
    }
    char line[512];
    int have_port = 0, have_ip = 0;
    while (fgets(line, sizeof line, f)) {
        char *s = trim(line);
        if (!*s || *s == '#') continue;
        char *eq = strchr(s, '=');
        if (!eq) {
            fprintf(stderr, "conf: %s: malformed line '%s' (expected KEY=VALUE)\n", path, s);
            fclose(f);
            return -1;
        }
        *eq = '\0';
        char *key = trim(s), *val = trim(eq + 1);
        if (!strcmp(key, "SERVER_PORT")) {
            char *end = NULL;
            long p = strtol(val, &end, 10);
            if (!*val || *end || p <= 0 || p > 65535) {
                fprintf(stderr, "conf: %s: bad SERVER_PORT '%s'\n", path, val);
                fclose(f);
                return -1;
            }
            out->server_port = (int)p;
            have_port = 1;
        } else if (!strcmp(key, "SERVER_IP")) {
            if (strlen(val) >= sizeof out->server_ip) {
                fclose(f);
                return -1;
            }
            strcpy(out->server_ip, val);
            have_ip = 1;
        }
    }
    fclose(f);
    if (!have_port || (need_ip && !have_ip)) {
        fprintf(stderr, "conf: %s: missing %s\n", path, have_port ? "SERVER_IP" : "SERVER_PORT");
        return -1;
    }
    return 0;
}
