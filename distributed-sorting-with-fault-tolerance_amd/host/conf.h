/* conf.h -- KEY=VALUE configuration files of the reference (server.conf, client.conf).
 *
 * Reference formats (read by read_conf_file, server.c:61-90 and client.c:15-54):
 *   server.conf:  SERVER_PORT=<port>
 *   client.conf:  SERVER_IP=<ipv4>      then    SERVER_PORT=<port>
 * The reference only accepts the keys in that order; this reader accepts them in any order,
 * ignores blank lines and '#' comments, and reports malformed files instead of continuing. */
#ifndef DSORT_CONF_H
#define DSORT_CONF_H

typedef struct dsort_conf {
    char server_ip[64];
    int server_port;
} dsort_conf;

/* Returns 0 on success, -1 if the file cannot be read or a value is malformed.
 * need_ip: SERVER_IP must be present (client.conf). */
int dsort_conf_read(const char *path, int need_ip, dsort_conf *out);

#endif
